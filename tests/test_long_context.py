"""Long context: Llama-3.1 RoPE scaling, 128k presets, the provider's context budget,
and (GPU) the prefill / decode attention kernels at 40k-100k tokens against an fp32 torch reference."""

import json
import math

import pytest
import torch

from llm_map_reduce_summarizer_amd.engine.config import get_model_config
from llm_map_reduce_summarizer_amd.ops import reference


def test_llama31_rope_scaling_rule():
    """Llama-3.1 "llama3" scaling: high frequencies (short wavelengths) kept, low frequencies / factor,
    the band between interpolated -- and plain RoPE without scaling."""
    plain = reference.rope_inv_freq(128, 500000.0)
    sc = reference.rope_inv_freq(128, 500000.0, (8.0, 1.0, 4.0, 8192))
    wl = 2 * math.pi / plain
    hi = wl < 8192 / 4.0
    lo = wl > 8192 / 1.0
    assert hi.any() and lo.any()
    assert torch.equal(sc[hi], plain[hi])
    assert torch.allclose(sc[lo], plain[lo] / 8.0)
    mid = ~(hi | lo)
    assert (sc[mid] <= plain[mid]).all() and (sc[mid] >= plain[mid] / 8.0).all()
    cs = reference.rope_cos_sin(16, 128, 500000.0, scaling=(8.0, 1.0, 4.0, 8192))
    assert cs.shape == (16, 64, 2)
    assert torch.allclose(cs[3, :, 0], torch.cos(3 * sc).float())


def test_llama31_presets_and_hf_roundtrip(tmp_path):
    from llm_map_reduce_summarizer_amd.engine.weights import config_from_hf
    c = get_model_config("llama3.1-8b")
    assert c.max_position == 131072 and c.rope_scaling == (8.0, 1.0, 4.0, 8192)
    assert get_model_config("llama3-8b").rope_scaling is None
    cfg = {"hidden_size": 4096, "intermediate_size": 14336, "num_hidden_layers": 32, "num_attention_heads": 32,
           "num_key_value_heads": 8, "vocab_size": 128256, "max_position_embeddings": 131072,
           "rope_theta": 500000.0, "rope_scaling": {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                   "high_freq_factor": 4.0,
                                                   "original_max_position_embeddings": 8192}}
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    got = config_from_hf(str(tmp_path))
    assert got.rope_scaling == (8.0, 1.0, 4.0, 8192) and got.max_position == 131072
    cfg["rope_scaling"] = {"rope_type": "yarn", "factor": 4.0}
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    with pytest.raises(ValueError):
        config_from_hf(str(tmp_path))


def test_provider_context_budget():
    """32k for the Llama-3 presets, the full 128k window for Llama-3.1, explicit value wins."""
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    assert LocalEngineProvider("llama3-8b").max_model_len == 32768
    assert LocalEngineProvider("llama3.1-8b").max_model_len == 131072
    assert LocalEngineProvider("llama3.1-8b", max_model_len=50000).max_model_len == 50000


def _ref_causal_rows(qkv, rows, hq, hkv, d, scale):
    """fp32 causal attention output of the given query rows of one packed sequence (torch, on qkv's device)."""
    g = hq // hkv
    q = qkv[rows, : hq * d].float().view(len(rows), hq, d)
    k = qkv[:, hq * d:(hq + hkv) * d].float().view(-1, hkv, d)
    v = qkv[:, (hq + hkv) * d:(hq + 2 * hkv) * d].float().view(-1, hkv, d)
    out = torch.empty(len(rows), hq, d, device=qkv.device)
    for i, r in enumerate(rows.tolist()):
        kk, vv = k[: r + 1], v[: r + 1]
        for h in range(hq):
            s = (kk[:, h // g] @ q[i, h]) * scale
            out[i, h] = torch.softmax(s, 0) @ vv[:, h // g]
    return out.view(len(rows), hq * d)


@pytest.mark.gpu
def test_attn_prefill_long_sequence():
    """One 40k-token causal sequence (hq=4, hkv=1): rows near the start, middle and end vs fp32."""
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = "cuda:0"
    T, hq, hkv, d = 40000, 4, 1, 128
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = (torch.randn(T, (hq + 2 * hkv) * d, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    cu = torch.tensor([0, T], dtype=torch.int32, device=dev)
    sc = 1.0 / math.sqrt(d)
    out = hip.attn_prefill(qkv, cu, hq, hkv, d, sc)
    rows = torch.tensor([0, 63, 64, 4095, 20011, 32768, 39998, 39999], device=dev)
    ref = _ref_causal_rows(qkv, rows, hq, hkv, d, sc)
    err = (out[rows].float() - ref).abs()
    assert err.max().item() < 3e-2 + 0, err.max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("paged", [False, True])
def test_attn_prefill_large_grid_kv_major(paged):
    """A packed prefill whose grid exceeds 2048 blocks runs in kv-head-major block order (attn_prefill.hip):
    3 x 6000 tokens at Llama-3-8B heads (2256 blocks), sampled rows of every sequence vs fp32; the paged
    variant reads the same keys from a shuffled page cache."""
    from llm_map_reduce_summarizer_amd import ops
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = "cuda:0"
    hq, hkv, d, L, nseq = 32, 8, 128, 6000, 3
    assert nseq * -(-L // hip.prefill_block_m(hq // hkv)) * hkv > 2048
    T = nseq * L
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = (torch.randn(T, (hq + 2 * hkv) * d, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
    sc = 1.0 / math.sqrt(d)
    pp = None
    if paged:
        npg = -(-L // 64)
        kc = torch.zeros(nseq * npg + 1, hkv, 64, d, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        perm = torch.randperm(nseq * npg, generator=g) + 1
        bt = perm.view(nseq, npg).to(torch.int32).to(dev)
        for s in range(nseq):
            rows = qkv[s * L:(s + 1) * L]
            kk = torch.zeros(npg * 64, hkv, d, dtype=torch.bfloat16, device=dev)
            vv = torch.zeros_like(kk)
            kk[:L] = rows[:, hq * d:(hq + hkv) * d].view(L, hkv, d)
            vv[:L] = rows[:, (hq + hkv) * d:].view(L, hkv, d)
            kc[bt[s].long()] = kk.view(npg, 64, hkv, d).transpose(1, 2)
            vc[bt[s].long()] = vv.view(npg, 64, hkv, d).transpose(1, 2)
        i32 = lambda x: torch.tensor(x, dtype=torch.int32, device=dev)  # noqa: E731
        pp = ops.PagedPrefill(bt, i32(list(range(nseq))), i32([0] * nseq), list(range(nseq)), [0] * nseq, kc, vc)
    out = hip.attn_prefill(qkv, cu, hq, hkv, d, sc, paged=pp)
    for s in range(nseq):
        rows = torch.tensor([0, 64, 2047, 4100, L - 1], device=dev)
        ref = _ref_causal_rows(qkv[s * L:(s + 1) * L], rows, hq, hkv, d, sc)
        err = (out[s * L + rows].float() - ref).abs()
        assert err.max().item() < 3e-2, (s, err.max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("ctx", [65536, 100001])
def test_attn_decode_long_context(ctx):
    """Decode attention over a 64k / 100k-token paged context with the engine's split plan vs fp32."""
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = "cuda:0"
    hq, hkv, d, page, B = 32, 8, 128, 64, 2
    npg = -(-ctx // page)
    n_pages = B * npg + 1
    g = torch.Generator(device="cpu").manual_seed(9)
    kc = (torch.randn(n_pages, hkv, page, d, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    vc = torch.randn(n_pages, hkv, page, d, generator=g).to(torch.bfloat16).to(dev)
    perm = (torch.randperm(n_pages - 1, generator=g) + 1).to(torch.int32)
    bt = perm[: B * npg].view(B, npg).contiguous().to(dev)
    pos = torch.tensor([ctx - 1, ctx // 3], dtype=torch.int32, device=dev)
    q = (torch.randn(B, (hq + 2 * hkv) * d, generator=g)).to(torch.bfloat16).to(dev)
    sc = 1.0 / math.sqrt(d)
    s, fused = hip.decode_attn_plan(B, hkv, 131072)
    ws = hip.DecodeWorkspace(B, hq, d, s, dev, hkv, fused_combine=fused)
    out = hip.attn_decode(q, kc, vc, bt, pos, hq, hkv, d, page, sc, workspace=ws)
    for b in range(B):
        n = int(pos[b]) + 1
        idx = bt[b, : -(-n // page)].long()
        k = kc[idx].permute(1, 0, 2, 3).reshape(hkv, -1, d)[:, :n].float()
        v = vc[idx].permute(1, 0, 2, 3).reshape(hkv, -1, d)[:, :n].float()
        qq = q[b, : hq * d].float().view(hq, d)
        for h in range(hq):
            p = torch.softmax((k[h // (hq // hkv)] @ qq[h]) * sc, 0)
            ref = p @ v[h // (hq // hkv)]
            err = (out[b, h * d:(h + 1) * d].float() - ref).abs().max().item()
            assert err < 2e-2, (b, h, err)
