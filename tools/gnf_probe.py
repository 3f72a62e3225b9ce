import sys, torch
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from oracle import autoencoder_ref
from panopticdiffusionmodels_amd import weights as W, _lib
from panopticdiffusionmodels_amd.libs.autoencoder import FrozenAutoencoderKL
lib = _lib.load()
def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm())
for init, seed in (("reference", 21), ("random", 3)):
    sd = W.make_state_dict(W.decoder_spec(ch=128, ch_mult=(1, 2, 4, 4), num_res_blocks=2), seed=seed, init=init)
    dd = dict(W.DECODER_DDCONFIG, ch=128, ch_mult=[1, 2, 4, 4], num_res_blocks=2)
    ae = FrozenAutoencoderKL(dd, 4, state_dict=sd, latent_size=32).to("cuda")
    z = torch.randn(2, 4, 32, 32, generator=torch.Generator().manual_seed(seed))
    fused = ae.decode(z.cuda()).cpu()
    lib.pdm_decoder_set_gn_fusion(0); sep = ae.decode(z.cuda()).cpu(); lib.pdm_decoder_set_gn_fusion(1)
    ref = autoencoder_ref.decode(sd, z[0:1])
    print(init, "fused-sep", rel(fused, sep), "fused-ref", rel(fused[0:1], ref), "sep-ref", rel(sep[0:1], ref), flush=True)
