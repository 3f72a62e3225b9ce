"""Network / sampler configurations of the five BASELINE configs (plain dicts, no ml_collections).

Shapes and hyper-parameters are restated from the reference's config files:
  * cifar10_uvit_small      configs/cifar10_uvit_small.py:36-47,55-61
  * imagenet256_uvit_large  configs/imagenet256_uvit_large.py:41-54,62-70
  * imagenet256_uvit_huge   configs/imagenet256_uvit_huge.py:41-55,62-70
  * imagenet512_uvit_huge   configs/imagenet512_uvit_huge.py:41-55,62-70
  * mscoco_uvit_small       configs/mscoco_uvit_small.py:41-55,63-70 (minus `patch_factor`,
    which libs/uvit_t2i.py:259-261 rejects)

`tiny_*` entries are the reduced shapes used for committed golden fixtures.
"""
import copy

CONFIGS = {
    "cifar10_uvit_small": dict(
        nnet=dict(name="uvit", img_size=32, patch_size=2, in_chans=3, embed_dim=512, depth=12,
                  num_heads=8, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=-1),
        z_shape=(3, 32, 32), front_end="dpm_solver_pytorch", cfg_scale=0.0, decode=False,
        sample_steps=50, eps=1e-4, mini_batch_size=4,
    ),
    "imagenet256_uvit_large": dict(
        nnet=dict(name="uvit", img_size=32, patch_size=2, in_chans=4, embed_dim=1024, depth=20,
                  num_heads=16, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=1001,
                  use_checkpoint=True),
        z_shape=(4, 32, 32), front_end="dpm_solver_pytorch", cfg_scale=0.4, decode=True,
        scale_factor=0.18215, sample_steps=50, eps=1e-4, mini_batch_size=50,
        # training (configs/imagenet256_uvit_large.py:19-40,57-60; train_ldm.py: sde.LSimple, noise_pred)
        train=dict(batch_size=1024, objective="sde", p_uncond=0.15, ema_rate=0.9999),
        optimizer=dict(name="adamw", lr=0.0002, weight_decay=0.03, betas=(0.99, 0.99)),
        lr_scheduler=dict(name="customized", warmup_steps=5000),
    ),
    "imagenet256_uvit_huge": dict(
        nnet=dict(name="uvit", img_size=32, patch_size=2, in_chans=4, embed_dim=1152, depth=28,
                  num_heads=16, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=1001,
                  use_checkpoint=True, conv=False),
        z_shape=(4, 32, 32), front_end="dpm_solver_pp", cfg_scale=0.4, decode=True,
        scale_factor=0.18215, sample_steps=50, mini_batch_size=50,
    ),
    "imagenet512_uvit_huge": dict(
        nnet=dict(name="uvit", img_size=64, patch_size=4, in_chans=4, embed_dim=1152, depth=28,
                  num_heads=16, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=1001,
                  use_checkpoint=True, conv=False),
        z_shape=(4, 64, 64), front_end="dpm_solver_pp", cfg_scale=0.7, decode=True,
        scale_factor=0.18215, sample_steps=50, mini_batch_size=50,
        precision="fp8",   # BASELINE configs[4]: "fp8 MFMA attention/MLP" (UViT.set_precision)
    ),
    "mscoco_uvit_small": dict(
        nnet=dict(name="uvit_t2i", img_size=32, in_chans=4, patch_size=2, embed_dim=512, depth=12,
                  num_heads=8, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, clip_dim=768,
                  num_clip_token=77, enable_panoptic=True, use_ground_truth=False, separate=True,
                  num_panoptic_class=8),
        z_shape=(4, 32, 32), front_end="dpm_solver_pp", cfg_scale=1.0, decode=True,
        scale_factor=0.23010, sample_steps=50, mini_batch_size=32, panoptic=True,
    ),
    # ---- tiny shapes for committed fixtures --------------------------------------------
    "tiny_uvit_cond": dict(  # Dh = 32, L = 2 + 64 tokens, class-conditional, conv final layer
        nnet=dict(name="uvit", img_size=16, patch_size=2, in_chans=4, embed_dim=64, depth=4,
                  num_heads=2, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=11),
        z_shape=(4, 16, 16), front_end="dpm_solver_pytorch", cfg_scale=0.4, decode=False,
        sample_steps=50, eps=1e-4, mini_batch_size=2,
    ),
    "tiny_uvit_h": dict(  # Dh = 72 (U-ViT-H head dim), patch 4, no conv
        nnet=dict(name="uvit", img_size=32, patch_size=4, in_chans=4, embed_dim=576, depth=2,
                  num_heads=8, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=11,
                  conv=False),
        z_shape=(4, 32, 32), front_end="dpm_solver_pp", cfg_scale=0.7, decode=False,
        sample_steps=50, mini_batch_size=2,
    ),
    "tiny_uvit_uncond": dict(  # CIFAR-style: no label token, pixel space
        nnet=dict(name="uvit", img_size=16, patch_size=2, in_chans=3, embed_dim=64, depth=2,
                  num_heads=2, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=-1),
        z_shape=(3, 16, 16), front_end="dpm_solver_pytorch", cfg_scale=0.0, decode=False,
        sample_steps=50, eps=1e-4, mini_batch_size=2,
    ),
    "tiny_uvit_train": dict(  # training-step fixtures: Dh = 64 (the attention backward), L = 2 + 64, conv
        nnet=dict(name="uvit", img_size=16, patch_size=2, in_chans=4, embed_dim=64, depth=2,
                  num_heads=1, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, num_classes=11),
        z_shape=(4, 16, 16), front_end="dpm_solver_pytorch", cfg_scale=0.4, decode=False,
        sample_steps=50, eps=1e-4, mini_batch_size=2,
        train=dict(batch_size=4, objective="discrete", p_uncond=0.15, ema_rate=0.9),
        optimizer=dict(name="adamw", lr=0.0002, weight_decay=0.03, betas=(0.99, 0.99)),
        lr_scheduler=dict(name="customized", warmup_steps=5),
    ),
    "tiny_uvit_train_uncond": dict(  # unconditional (no label token), qkv bias, no final conv
        nnet=dict(name="uvit", img_size=16, patch_size=2, in_chans=3, embed_dim=64, depth=2,
                  num_heads=1, mlp_ratio=4, qkv_bias=True, mlp_time_embed=False, num_classes=-1, conv=False),
        z_shape=(3, 16, 16), front_end="dpm_solver_pytorch", cfg_scale=0.0, decode=False,
        sample_steps=50, eps=1e-4, mini_batch_size=2,
        train=dict(batch_size=4, objective="sde", p_uncond=0.0, ema_rate=0.9),
        optimizer=dict(name="adamw", lr=0.0002, weight_decay=0.03, betas=(0.99, 0.999)),
        lr_scheduler=dict(name="customized", warmup_steps=-1),
    ),
    "tiny_t2i": dict(  # panoptic co-generation, separate streams
        nnet=dict(name="uvit_t2i", img_size=16, in_chans=4, patch_size=2, embed_dim=64, depth=2,
                  num_heads=2, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, clip_dim=64,
                  num_clip_token=5, enable_panoptic=True, use_ground_truth=False, separate=True,
                  num_panoptic_class=8),
        z_shape=(4, 16, 16), front_end="dpm_solver_pp", cfg_scale=1.0, decode=False,
        sample_steps=50, mini_batch_size=2, panoptic=True,
    ),
    "tiny_uvit_train_h": dict(  # training fixtures at head dim 72 (U-ViT-H): 8 heads x 72, L = 2 + 64, conv
        nnet=dict(name="uvit", img_size=16, patch_size=2, in_chans=4, embed_dim=576, depth=2,
                  num_heads=8, mlp_ratio=2, qkv_bias=False, mlp_time_embed=False, num_classes=11),
        z_shape=(4, 16, 16), front_end="dpm_solver_pp", cfg_scale=0.4, decode=False,
        sample_steps=50, mini_batch_size=2,
        train=dict(batch_size=4, objective="discrete", p_uncond=0.15, ema_rate=0.9),
        optimizer=dict(name="adamw", lr=0.0002, weight_decay=0.03, betas=(0.99, 0.99)),
        lr_scheduler=dict(name="customized", warmup_steps=5),
    ),
    "tiny_t2i_train": dict(  # panoptic t2i training fixtures: Dh = 64, the full token counts (Lx 334, Lm 590), conv
        nnet=dict(name="uvit_t2i", img_size=32, in_chans=4, patch_size=2, embed_dim=64, depth=2,
                  num_heads=1, mlp_ratio=4, qkv_bias=False, mlp_time_embed=False, clip_dim=64,
                  num_clip_token=77, enable_panoptic=True, use_ground_truth=False, separate=True,
                  num_panoptic_class=8),
        z_shape=(4, 32, 32), front_end="dpm_solver_pp", cfg_scale=1.0, decode=False,
        sample_steps=50, mini_batch_size=2, panoptic=True,
        train=dict(batch_size=2, objective="discrete", p_uncond=0.0, ema_rate=0.9),
        optimizer=dict(name="adamw", lr=0.0002, weight_decay=0.03, betas=(0.99, 0.99)),
        lr_scheduler=dict(name="customized", warmup_steps=-1),
    ),
}


def get_config(name):
    if name not in CONFIGS:
        raise KeyError(f"unknown config {name!r}; known: {sorted(CONFIGS)}")
    return copy.deepcopy(CONFIGS[name])


def nnet_kwargs(name):
    """The `config.nnet` dict as `utils.get_nnet(**config.nnet)` receives it."""
    return get_config(name)["nnet"]
