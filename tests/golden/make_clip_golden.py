"""Generate tests/golden/clip_golden.npz: the t2i conditioning producer's golden vectors (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_clip_golden.py [/root/reference]

libs/clip.py:13-38 (FrozenCLIPEmbedder) wraps transformers' CLIPTextModel and returns
`transformer(input_ids=tokens).last_hidden_state` (libs/clip.py:33-36).  `from_pretrained` needs the network
(openai/clip-vit-large-patch14), so the model is built from a CLIPTextConfig with seeded random weights (two tiny
configs: head dim 32 and 64) and called exactly like libs/clip.py does.  The reference module itself is imported
to confirm that its `transformer` is transformers' CLIPTextModel.  Stored: the state_dict, the token ids and
last_hidden_state.  Nothing here runs on the GPU box; the .npz is data.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

CONFIGS = {
    "clip_dh32": dict(vocab_size=256, hidden_size=64, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=2, max_position_embeddings=77),
    "clip_dh64": dict(vocab_size=256, hidden_size=128, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, max_position_embeddings=77),
}


def main(ref):
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    import libs.clip as rclip   # noqa: F401  (the reference module: FrozenCLIPEmbedder over CLIPTextModel)
    from transformers import CLIPTextConfig, CLIPTextModel
    assert rclip.CLIPTextModel is CLIPTextModel
    out = {}
    for name, kw in CONFIGS.items():
        torch.manual_seed(1234)
        cfg = CLIPTextConfig(hidden_act="quick_gelu", layer_norm_eps=1e-5, bos_token_id=0, eos_token_id=1,
                             pad_token_id=1, **kw)
        model = CLIPTextModel(cfg).eval()
        with torch.no_grad():   # non-trivial LayerNorm affines and biases (the init leaves them 1 / 0)
            for k, v in model.state_dict().items():
                if "norm" in k or k.endswith(".bias"):
                    v.copy_(torch.randn_like(v) * 0.2 + (1.0 if "norm" in k and k.endswith(".weight") else 0.0))
        ids = torch.randint(0, kw["vocab_size"], (3, 77), generator=torch.Generator().manual_seed(7))
        ids[2, 20:] = 1   # a padded prompt: eos / pad tail, as the tokenizer's padding="max_length"
        with torch.no_grad():
            z = model(input_ids=ids).last_hidden_state
        for k, v in model.state_dict().items():
            out[f"{name}/sd/{k}"] = v.numpy()
        out[f"{name}/ids"] = ids.numpy()
        out[f"{name}/out"] = z.numpy()
        out[f"{name}/heads"] = np.array(kw["num_attention_heads"])
    np.savez_compressed(os.path.join(HERE, "clip_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "clip_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
