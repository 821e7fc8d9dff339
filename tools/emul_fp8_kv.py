#!/usr/bin/env python3
"""CPU emulation of the fp8 KV cache formats on the parity checkpoint of tests/test_forward_parity_gpu.py
(Llama-3-8B dims, 2 layers, peaked attention): max relative L2 error of the last 8 logit rows against the
unquantised fp32 forward with K and V, K only or V only stored as e4m3 rows with power-of-two row scales
(kv8.h)."""
import math, os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, ROOT)
import test_forward_parity_gpu as P
from llm_map_reduce_summarizer_amd.engine.config import get_model_config
torch.set_num_threads(8)
cfg = get_model_config("llama3-8b", n_layers=2)
ck = P._checkpoint(cfg, 4)
ones = torch.ones(cfg.hidden, dtype=torch.bfloat16)
for i in range(2):
    for k in ("input_layernorm.weight", "post_attention_layernorm.weight"):
        ck["model.layers.%d.%s" % (i, k)] = ones
ck["model.norm.weight"] = ones
def q_row_pow2(x):
    amax = x.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    s = 2.0 ** torch.ceil(torch.log2(amax / 448))
    return (x / s).to(torch.float8_e4m3fn).float() * s
def fwd(tokens, qk, qv):
    H, hd, hq, hk = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
    f = lambda k: ck[k].float()
    n = len(tokens); x = f("model.embed_tokens.weight")[torch.tensor(tokens)]
    ang = torch.arange(n, dtype=torch.float64)[:, None] * P._inv_freq(cfg)[None]
    cos = torch.cat([ang.cos(), ang.cos()], -1).float()[:, None]; sin = torch.cat([ang.sin(), ang.sin()], -1).float()[:, None]
    rope = lambda t: t * cos + torch.cat([-t[..., hd // 2:], t[..., :hd // 2]], -1) * sin
    mask = torch.full((n, n), float("-inf")).triu(1)
    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        h = P._rms(x, 1.0, cfg.rms_eps)
        q = rope((h @ f(p + "self_attn.q_proj.weight").t()).view(n, hq, hd))
        k = rope((h @ f(p + "self_attn.k_proj.weight").t()).view(n, hk, hd))
        v = (h @ f(p + "self_attn.v_proj.weight").t()).view(n, hk, hd)
        if qk: k = q_row_pow2(k)
        if qv: v = q_row_pow2(v)
        g = hq // hk
        s = torch.einsum("nhd,mhd->hnm", q, k.repeat_interleave(g, 1)) / math.sqrt(hd) + mask
        out = torch.einsum("hnm,mhd->nhd", torch.softmax(s, -1), v.repeat_interleave(g, 1))
        x = x + out.reshape(n, hq * hd) @ f(p + "self_attn.o_proj.weight").t()
        h = P._rms(x, 1.0, cfg.rms_eps)
        a = torch.nn.functional.silu(h @ f(p + "mlp.gate_proj.weight").t()) * (h @ f(p + "mlp.up_proj.weight").t())
        x = x + a @ f(p + "mlp.down_proj.weight").t()
    h = P._rms(x, 1.0, cfg.rms_eps)
    return (h @ f("model.embed_tokens.weight").t())[-8:]
toks = P._prompts((333,), 6)[0]
ref = fwd(toks, False, False)
def err(y): return float(((y - ref).norm(dim=-1) / ref.norm(dim=-1)).max())
print("K+V fp8 %.4f" % err(fwd(toks, True, True)))
print("K fp8 only %.4f" % err(fwd(toks, True, False)))
print("V fp8 only %.4f" % err(fwd(toks, False, True)))
