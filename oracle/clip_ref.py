"""ORACLE (test infrastructure): fp32 CPU restatement of the t2i conditioning producer.

libs/clip.py:13-38 `FrozenCLIPEmbedder.encode(text)` = `CLIPTextModel(input_ids=tokens).last_hidden_state`
(tokens from CLIPTokenizer, padding="max_length", max_length=77).  The arithmetic lives in the third-party
`transformers` package (not vendored in the reference, no pinned version; this container has 5.15.0,
`transformers/models/clip/modeling_clip.py`): CLIPTextEmbeddings, CLIPEncoderLayer (pre-LN, causal
CLIPAttention, CLIPMLP with quick_gelu), final_layer_norm.  Restated here from that published algorithm and
pinned against CLIPTextModel itself (tests/golden/make_clip_golden.py -> tests/golden/clip_golden.npz,
tests/test_clip.py).  Parameters: a CLIPTextModel state_dict (keys without the "text_model." prefix).
"""
import torch
import torch.nn.functional as F


def clip_text_forward(sd, ids, heads, eps=1e-5):
    """ids int64 [B, L] -> last_hidden_state fp32 [B, L, width]."""
    sd = {k: v.float() for k, v in sd.items()}
    B, L = ids.shape
    # CLIPTextEmbeddings: token_embedding(ids) + position_embedding(arange(L))
    x = sd["embeddings.token_embedding.weight"][ids] + sd["embeddings.position_embedding.weight"][:L][None]
    D = x.shape[-1]
    Dh = D // heads
    causal = torch.full((L, L), float("-inf")).triu(1)
    n = 0
    while f"encoder.layers.{n}.layer_norm1.weight" in sd:
        p = f"encoder.layers.{n}"
        # CLIPEncoderLayer: x = x + self_attn(layer_norm1(x), causal); x = x + mlp(layer_norm2(x))
        h = F.layer_norm(x, (D,), sd[p + ".layer_norm1.weight"], sd[p + ".layer_norm1.bias"], eps)

        def proj(name, t):
            return F.linear(t, sd[f"{p}.self_attn.{name}.weight"], sd[f"{p}.self_attn.{name}.bias"])

        q = proj("q_proj", h).reshape(B, L, heads, Dh).transpose(1, 2)
        k = proj("k_proj", h).reshape(B, L, heads, Dh).transpose(1, 2)
        v = proj("v_proj", h).reshape(B, L, heads, Dh).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) * Dh ** -0.5 + causal
        a = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, D)
        x = x + proj("out_proj", a)
        h = F.layer_norm(x, (D,), sd[p + ".layer_norm2.weight"], sd[p + ".layer_norm2.bias"], eps)
        h = F.linear(h, sd[p + ".mlp.fc1.weight"], sd[p + ".mlp.fc1.bias"])
        h = h * torch.sigmoid(1.702 * h)   # quick_gelu (transformers QuickGELUActivation)
        x = x + F.linear(h, sd[p + ".mlp.fc2.weight"], sd[p + ".mlp.fc2.bias"])
        n += 1
    return F.layer_norm(x, (D,), sd["final_layer_norm.weight"], sd["final_layer_norm.bias"], eps)
