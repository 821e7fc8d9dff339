"""Full-forward parity on the GPU: the engine's HIP prefill and decode logits of a Llama-3-8B-shaped
model (real dims, 2 layers, random HF-layout weights with NON-unit RMSNorm gains) against an
independent textbook fp32 forward written here from the checkpoint tensors -- separate q/k/v/o and
gate/up/down matrices, explicit gains, HF rotate-half RoPE with its own Llama-3.1 scaling formula.

What it guards (a bug shared by prefill and decode passes every self-consistency test): the loader's
gain folding and gate/up interleave, the RoPE (and RoPE-scaling) table, the fused QKV / SwiGLU /
split-K epilogues, the deferred decode norm, paged KV and chunked prefill, and the fp8 row-scale
order (fp8 is compared with the textbook forward of the dequantised engine weights).

The engine replaces the reference's hosted LLM call (/root/reference/llm_executor.py:283-297), so
this is the numerics contract of that black box."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from llm_map_reduce_summarizer_amd.engine import weights as W  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams  # noqa: E402


class _Mem:
    def __init__(self, d):
        self.d = d

    def get_tensor(self, k):
        return self.d[k]


def _checkpoint(cfg, seed, tied=True):
    """HF-layout random tensors (bf16, CPU) with gains ~ 1 +- 0.2.  q / k projections get std
    2.5 / sqrt(hidden): attention scores of std ~6, so attention is peaked and position-sensitive (with
    near-uniform random attention a wrong RoPE table would hardly move the logits)."""
    g = torch.Generator().manual_seed(seed)
    H, hd, F = cfg.hidden, cfg.head_dim, cfg.ffn
    qk = 2.5 / math.sqrt(H)

    def rn(*shape, std=0.02):
        return (torch.randn(*shape, generator=g) * std).to(torch.bfloat16)

    def gain():
        return (1.0 + 0.2 * torch.randn(H, generator=g)).to(torch.bfloat16)
    d = {"model.embed_tokens.weight": rn(cfg.vocab_size, H, std=1.0), "model.norm.weight": gain()}
    if not tied:
        d["lm_head.weight"] = rn(cfg.vocab_size, H)
    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        d[p + "input_layernorm.weight"] = gain()
        d[p + "post_attention_layernorm.weight"] = gain()
        d[p + "self_attn.q_proj.weight"] = rn(cfg.n_heads * hd, H, std=qk)
        d[p + "self_attn.k_proj.weight"] = rn(cfg.n_kv_heads * hd, H, std=qk)
        d[p + "self_attn.v_proj.weight"] = rn(cfg.n_kv_heads * hd, H)
        d[p + "self_attn.o_proj.weight"] = rn(H, cfg.n_heads * hd)
        d[p + "mlp.gate_proj.weight"] = rn(F, H)
        d[p + "mlp.up_proj.weight"] = rn(F, H)
        d[p + "mlp.down_proj.weight"] = rn(H, F)
    return d


def _inv_freq(cfg):
    """HF Llama rotary frequencies, with the 'llama3' scaling rule written out independently."""
    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    if cfg.rope_scaling:
        factor, lo, hi, old = cfg.rope_scaling
        out = []
        for f in inv.tolist():
            wl = 2 * math.pi / f
            if wl < old / hi:
                out.append(f)
            elif wl > old / lo:
                out.append(f / factor)
            else:
                s = (old / wl - lo) / (hi - lo)
                out.append((1 - s) * f / factor + s * f)
        inv = torch.tensor(out, dtype=torch.float64)
    return inv


def _rms(x, g, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * g


def _textbook_logits(T, cfg, tokens, dev):
    """fp32 logits [len(tokens), vocab] of a plain causal Llama forward over ``tokens``."""
    H, hd, hq, hk = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
    f = lambda k: T[k].to(dev, torch.float32)  # noqa: E731
    ids = torch.tensor(tokens, device=dev)
    n = len(tokens)
    x = f("model.embed_tokens.weight")[ids]
    ang = torch.arange(n, dtype=torch.float64)[:, None] * _inv_freq(cfg)[None]
    cos = torch.cat([ang.cos(), ang.cos()], -1).float().to(dev)[:, None]
    sin = torch.cat([ang.sin(), ang.sin()], -1).float().to(dev)[:, None]

    def rope(t):
        t1, t2 = t[..., :hd // 2], t[..., hd // 2:]
        return t * cos + torch.cat([-t2, t1], -1) * sin
    mask = torch.full((n, n), float("-inf"), device=dev).triu(1)
    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        h = _rms(x, f(p + "input_layernorm.weight"), cfg.rms_eps)
        q = rope((h @ f(p + "self_attn.q_proj.weight").t()).view(n, hq, hd))
        k = rope((h @ f(p + "self_attn.k_proj.weight").t()).view(n, hk, hd))
        v = (h @ f(p + "self_attn.v_proj.weight").t()).view(n, hk, hd)
        out = torch.empty(n, hq, hd, device=dev)
        for hh in range(hq):
            kv = hh // (hq // hk)
            s = (q[:, hh] @ k[:, kv].t()) / math.sqrt(hd) + mask
            out[:, hh] = torch.softmax(s, -1) @ v[:, kv]
        x = x + out.reshape(n, hq * hd) @ f(p + "self_attn.o_proj.weight").t()
        h = _rms(x, f(p + "post_attention_layernorm.weight"), cfg.rms_eps)
        a = torch.nn.functional.silu(h @ f(p + "mlp.gate_proj.weight").t()) * (h @ f(p + "mlp.up_proj.weight").t())
        x = x + a @ f(p + "mlp.down_proj.weight").t()
    h = _rms(x, f("model.norm.weight"), cfg.rms_eps)
    lm = f("lm_head.weight") if "lm_head.weight" in T else f("model.embed_tokens.weight")
    return h @ lm.t()


def _engine_run(monkeypatch, cfg, ckpt, prompts, new, **kw):
    """Greedy generate of ``new`` tokens; returns (token ids per prompt, logits rows per prompt: the
    prefill row then one row per decode step), recorded at the sampler."""
    index = {k: "mem" for k in ckpt}
    monkeypatch.setattr(W, "_open_shards", lambda path: (index, {"mem": _Mem(ckpt)}))
    eng = LLMEngine(cfg, device="cuda:0", weights_path="mem", use_graphs=False, max_num_seqs=8, sync_every=64,
                    **kw)
    rec = []
    orig = eng._sample

    def spy(logits, view):
        rec.append(logits.float().clone())
        orig(logits, view)
    eng._sample = spy
    outs = eng.generate(prompts, [SamplingParams(new, 0.0, 0)] * len(prompts), ignore_eos=True)
    torch.cuda.synchronize()
    # slot order = admission order (longest first, stable) for the prefill pass(es) and every step
    order = sorted(range(len(prompts)), key=lambda i: -len(prompts[i]))
    pre = torch.cat([r for r in rec[:len(rec) - (new - 1)]])  # prefill pass(es): one row per prompt
    steps = rec[len(rec) - (new - 1):]
    rows = {}
    for slot, i in enumerate(order):
        rows[i] = [pre[slot]] + [s[slot] for s in steps]
    model = eng.model
    del eng
    return [o.token_ids for o in outs], rows, model


def _compare(cfg, ref_ckpt, prompts, toks, rows, rel_tol, dev, min_exact=0.9, per_prompt=None):
    errs, exact, total = [], 0, 0
    for i, p in enumerate(prompts):
        ref = _textbook_logits(ref_ckpt, cfg, p + toks[i][:-1], dev)[len(p) - 1:]  # teacher-forced rows
        for r, got in zip(ref, rows[i]):
            d = (got - r).norm() / r.norm()
            errs.append(float(d))
            if per_prompt is not None:
                per_prompt.setdefault(i, []).append(float(d))
            # top-1: exact, or a near-tie of the reference (within a few error-sizes of its max)
            a = int(got.argmax())
            exact += a == int(r.argmax())
            total += 1
            tie = 4 * float((got - r).abs().max())
            assert float(r[a]) >= float(r.max()) - tie, (i, a, int(r.argmax()))
    assert max(errs) <= rel_tol, errs
    assert exact >= min_exact * total, (exact, total)
    return max(errs), exact, total


# Relative L2 error bounds of a logits row.  The engine keeps activations in bf16 (the textbook forward
# in fp32): with the peaked attention of these checkpoints the CPU reference ops in bf16 land at
# 0.9-3.5 % on the same model and prompts (the GPU at 0.7-4.2 %), while a wrong RoPE table puts rows
# at 30 %+ -- the bounds sit between.  fp8 adds the e4m3 activation rounding of the prefill GEMMs.
BF16_TOL = 0.07
# fp8: prefill GEMMs round the activations to e4m3 per row (3 mantissa bits, ~2.3 % RMS per element);
# the peaked attention amplifies that on prefilled rows -- 20-26 % when the QKV input was single-term (round
# 3).  The QKV input is now two-term fp8 (hi + lo / 16, ops.hip.rmsnorm_fp8 split): measured 9.5-10.9 % on
# prefilled rows, 1-7 % on decode rows (profiles/r4_gpu_tests_fp8kv_twoterm.txt; the CPU emulation of the
# same checkpoint predicts 10.1 %, profiles/r4_fp8_activation_emulation.txt).  The W8A16 decode kernels keep
# bf16 activations (a one-token prompt's rows: 1-7 %).  A wrong row-scale order or a lost lo half is O(0.2+).
FP8_TOL = 0.15
FP8_MIN_EXACT = 0.9
FP8_W8A16_TOL = 0.1


def _prompts(lengths, seed):
    g = torch.Generator().manual_seed(seed)
    return [[128000] + torch.randint(5, 120000, (n - 1,), generator=g).tolist() for n in lengths]


def test_llama3_8b_dims_bf16_parity(monkeypatch):
    cfg = get_model_config("llama3-8b", n_layers=2)
    ckpt = _checkpoint(cfg, 1)
    prompts = _prompts((1, 17, 300, 129, 1000, 64, 513), 3)  # packed ragged prefill, B = 7 decode
    toks, rows, _ = _engine_run(monkeypatch, cfg, ckpt, prompts, 4, max_model_len=2048, kv_pages=256)
    err, exact, total = _compare(cfg, ckpt, prompts, toks, rows, BF16_TOL, torch.device("cuda:0"))
    print("bf16 parity: max rel err %.4f, top-1 %d/%d" % (err, exact, total))


def test_llama31_rope_scaled_chunked_prefill_parity(monkeypatch):
    """Llama-3.1 RoPE scaling at ~9k positions (the scaled low frequencies matter there), prefilled in
    4096-token slices through the paged cache, then 3 decode steps."""
    cfg = get_model_config("llama3.1-8b", n_layers=2)
    ckpt = _checkpoint(cfg, 2, tied=False)
    prompts = _prompts((9000, 8193), 5)
    toks, rows, _ = _engine_run(monkeypatch, cfg, ckpt, prompts, 4, max_model_len=10240, kv_pages=400)
    err, exact, total = _compare(cfg, ckpt, prompts, toks, rows, BF16_TOL, torch.device("cuda:0"))
    print("llama3.1 parity: max rel err %.4f, top-1 %d/%d" % (err, exact, total))


def test_llama3_8b_dims_fp8_parity(monkeypatch):
    """fp8 weights (OCP e4m3fn, per-row scales): engine logits vs the textbook forward of the engine's
    own dequantised weights (gains already folded in: unit gains in the reference checkpoint)."""
    cfg = get_model_config("llama3-8b", n_layers=2)
    ckpt = _checkpoint(cfg, 4)
    prompts = _prompts((1, 40, 333, 700, 96), 6)
    toks, rows, model = _engine_run(monkeypatch, cfg, ckpt, prompts, 4, max_model_len=2048, kv_pages=256,
                                    weight_dtype="fp8")
    hd, qs, ks = cfg.head_dim, cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
    ones = torch.ones(cfg.hidden, dtype=torch.bfloat16)
    ref = {"model.embed_tokens.weight": ckpt["model.embed_tokens.weight"], "model.norm.weight": ones,
           "lm_head.weight": model.lm_head.dequant(torch.float32)}
    from llm_map_reduce_summarizer_amd.ops.reference import split_gate_up
    for i, lw in enumerate(model.layers):
        p = "model.layers.%d." % i
        qkv = lw.wqkv.dequant(torch.float32)
        ref[p + "self_attn.q_proj.weight"] = qkv[:qs]
        ref[p + "self_attn.k_proj.weight"] = qkv[qs:qs + ks]
        ref[p + "self_attn.v_proj.weight"] = qkv[qs + ks:]
        ref[p + "self_attn.o_proj.weight"] = lw.wo.dequant(torch.float32)
        gg, uu = split_gate_up(lw.wgu.dequant(torch.float32).t())
        ref[p + "mlp.gate_proj.weight"], ref[p + "mlp.up_proj.weight"] = gg.t(), uu.t()
        ref[p + "mlp.down_proj.weight"] = lw.wdown.dequant(torch.float32)
        ref[p + "input_layernorm.weight"] = ones
        ref[p + "post_attention_layernorm.weight"] = ones
    assert hd == 128
    pp = {}
    err, exact, total = _compare(cfg, ref, prompts, toks, rows, FP8_TOL, torch.device("cuda:0"),
                                 min_exact=FP8_MIN_EXACT, per_prompt=pp)
    print("fp8 parity: max rel err %.4f, top-1 %d/%d, per prompt %s" % (
        err, exact, total, {i: [round(x, 3) for x in v] for i, v in pp.items()}))
    assert max(pp[0]) <= FP8_W8A16_TOL, pp[0]  # the 1-token prompt: weight-only fp8 (W8A16) kernels throughout


# fp8 KV cache (e4m3 rows, power-of-two row scales: ~2.7 % RMS per element, kv8.h): every row here attends
# over dequantised K/V (the 1300-token prompt makes every prefill pass chunked, through the cache), and the
# peaked attention of this checkpoint (score std ~6) amplifies the K error like it amplifies fp8 activations
# (single-term: 24 %): measured 13-22 % on prompts with history, 3.8 % on the one-token prompt, top-1 20/20
# (profiles/r4_gpu_tests_fp8kv_twoterm.txt, r5_parity_bf16_fp8_fp8kv_fp8v.txt).  Above the 0.15 a KV variant
# must meet, so the CLI / bench offer only fp8v (V fp8, K bf16: 7.95 %) below.
FP8_KV_TOL = 0.25


def test_llama3_8b_dims_fp8_kv_parity(monkeypatch):
    """kv_dtype="fp8" (K and V fp8; an engine format the CLI does not offer, see FP8_KV_TOL): packed + chunked
    prefill (slices attend to their prefix through the fp8 cache) and
    decode over the fp8 cache, vs the textbook fp32 forward (bf16 weights)."""
    cfg = get_model_config("llama3-8b", n_layers=2)
    ckpt = _checkpoint(cfg, 7)
    prompts = _prompts((1, 40, 333, 700, 1300), 8)
    toks, rows, _ = _engine_run(monkeypatch, cfg, ckpt, prompts, 4, max_model_len=2048, kv_pages=256,
                                kv_dtype="fp8", prefill_chunk=512)
    pp = {}
    err, exact, total = _compare(cfg, ckpt, prompts, toks, rows, FP8_KV_TOL, torch.device("cuda:0"),
                                 min_exact=0.8, per_prompt=pp)
    print("fp8 KV parity: max rel err %.4f, top-1 %d/%d, per prompt %s" % (
        err, exact, total, {i: [round(x, 3) for x in v] for i, v in pp.items()}))


# fp8 V cache, bf16 K ("fp8v"): V rows e4m3 with power-of-two row scales, K bf16 -- the
# attention probabilities weight the V rounding (~2.7 % RMS per element) linearly instead of the scores
# amplifying it (the CPU emulation of this checkpoint: 6.3 % vs K+V 20 %, profiles/r4_fp8_kv_emulation.txt).
FP8V_KV_TOL = 0.10
FP8V_MIN_EXACT = 0.9


def test_llama3_8b_dims_fp8v_kv_parity(monkeypatch):
    """--kv-dtype fp8v: packed + chunked prefill through the bf16-K / fp8-V cache and decode over it, vs the
    textbook fp32 forward (bf16 weights), with the bound the verdict set for a KV variant worth offering."""
    cfg = get_model_config("llama3-8b", n_layers=2)
    ckpt = _checkpoint(cfg, 7)
    prompts = _prompts((1, 40, 333, 700, 1300), 8)
    toks, rows, model = _engine_run(monkeypatch, cfg, ckpt, prompts, 4, max_model_len=2048, kv_pages=256,
                                    kv_dtype="fp8v", prefill_chunk=512)
    pp = {}
    err, exact, total = _compare(cfg, ckpt, prompts, toks, rows, FP8V_KV_TOL, torch.device("cuda:0"),
                                 min_exact=FP8V_MIN_EXACT, per_prompt=pp)
    print("fp8v KV parity: max rel err %.4f, top-1 %d/%d, per prompt %s" % (
        err, exact, total, {i: [round(x, 3) for x in v] for i, v in pp.items()}))
