"""ORACLE — test infrastructure only.

A PyTorch-CPU fp32 functional restatement of the reference's sampling hot path
(yinghanlong/PanopticDiffusionModels @ 2025-07-25): U-ViT / U-ViT-t2i forward, the two DPM-Solver
front-ends, classifier-free guidance, the KL-f8 decoder and the analog-bit codecs.  Each function cites
the reference file:line it restates.

Pinning: every function here is checked against golden vectors produced by importing the reference
itself in the build container (tests/golden/make_golden.py -> tests/golden/*.npz,
tests/test_oracle_golden.py).  The reference never travels to the GPU box; the fixtures do.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and only
as the checker / the timed CPU baseline.  The product path (panopticdiffusionmodels_amd) never
imports it and fails loudly when its HIP library is missing.
"""
