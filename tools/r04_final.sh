#!/bin/bash
# End-of-session evidence: the L/2 forward A/B vs the pre-grouping lib, then the full validation (tools/r04_validate.sh).
bash tools/r04_pair2.sh ${2:-r04q} || exit $?
bash tools/r04_validate.sh ${1:-r04w}
