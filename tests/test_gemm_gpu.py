"""Large-M MFMA GEMM (csrc/kernels/gemm.hip) vs a plain PyTorch fp32 reference.

Covers ragged M (tiles past M), N tails (a vocab shard that is not a multiple of 256),
strided activations, both epilogues (LDS-staged 16-B row stores for aligned outputs, register
stores for outputs that are not 16-B aligned), the fused SwiGLU epilogue, and the fp8
(OCP e4m3fn, block-scaled MFMA with unit scales) path against the dequantised fp32 product.
Data is asymmetric random (an output transpose or a row/column swap would not pass).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

from llm_map_reduce_summarizer_amd.ops import hip, reference  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402

DEV = "cuda:0"


def _rand(*shape, scale=1.0, seed=0, offset=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale + offset).to(torch.bfloat16).to(DEV)


def _check(out, ref, tol=2e-2):
    out, ref = out.float(), ref.float()
    err = (out - ref).abs()
    bound = tol * (ref.abs() + ref.abs().mean())
    bad = int((err > bound).sum())
    assert bad == 0, "max err %.4g (%d bad of %d), ref mean |x| %.4g" % (err.max(), bad, out.numel(),
                                                                         ref.abs().mean())


@pytest.mark.parametrize("M,N,K", [(65, 256, 128), (1000, 1280, 4096), (4097, 6144, 4096),
                                   (300, 16032, 1024), (16384 + 13, 4096, 1024), (257, 4096, 14336)])
@pytest.mark.parametrize("aligned", [True, False])
def test_gemm_bf16(M, N, K, aligned):
    x = _rand(M, K, seed=1, scale=0.5, offset=0.05)
    w = _rand(N, K, seed=2, scale=0.02, offset=0.001)
    ref = x.float() @ w.float().t()
    if aligned:
        out = hip.gemm(x, w)
    else:  # an 8-byte (not 16-byte) aligned output view: the register-store epilogue
        big = torch.zeros(M, N + 8, dtype=torch.bfloat16, device=DEV)
        out = hip.gemm(x, w, out=big[:, 4:4 + N])
    torch.cuda.synchronize()
    _check(out, ref)


def test_gemm_bf16_identity_asymmetric():
    """A = I exposes a transposed store; W asymmetric so a row/col swap shows."""
    K = 256
    x = torch.eye(K, dtype=torch.bfloat16, device=DEV)
    w = (torch.arange(512 * K, device=DEV, dtype=torch.float32).reshape(512, K) % 97 - 48).to(torch.bfloat16)
    out = hip.gemm(x, w)
    torch.cuda.synchronize()
    assert torch.equal(out.float(), w.float().t()), "C = I . W^T must equal W^T exactly"


def test_gemm_strided_input_and_out():
    M, K, N = 700, 1024, 512
    big = _rand(M, K + 64, seed=3, scale=0.3)
    x = big[:, 32:32 + K]
    w = _rand(N, K, seed=4, scale=0.05)
    for off in (0, 4):  # 16-B aligned view (LDS epilogue) and 8-B aligned view (register epilogue)
        out_big = torch.zeros(M, N + 16, dtype=torch.bfloat16, device=DEV)
        hip.gemm(x, w, out=out_big[:, off:off + N])
        torch.cuda.synchronize()
        _check(out_big[:, off:off + N], x.float() @ w.float().t())
        assert float(out_big[:, N + off:].abs().max()) == 0.0 and float(out_big[:, :off].abs().max() if off else 0) == 0.0, \
            "wrote outside the output view"


@pytest.mark.parametrize("M", [100, 3000])
def test_gemm_swiglu(M):
    K, F = 4096, 1792
    x = _rand(M, K, seed=5, scale=0.5)
    wg, wu = _rand(F, K, seed=6, scale=0.03), _rand(F, K, seed=7, scale=0.03)
    wgu = reference.interleave_gate_up(wg, wu).contiguous()
    out = hip.gemm(x, wgu, swiglu=True)
    torch.cuda.synchronize()
    g, u = x.float() @ wg.float().t(), x.float() @ wu.float().t()
    _check(out, torch.nn.functional.silu(g) * u, tol=3e-2)


@pytest.mark.parametrize("M,N,K", [(77, 1280, 8192), (2049, 7168, 8192), (513, 16032, 1024)])
@pytest.mark.parametrize("swiglu", [False, True])
def test_gemm_fp8(M, N, K, swiglu):
    x = _rand(M, K, seed=8, scale=0.5, offset=0.02)
    w = Fp8Weight.quantize(_rand(N, K, seed=9, scale=0.02))
    xq, xs = hip.quant_fp8_rows(x)
    out = hip.gemm_fp8(xq, xs, w, swiglu=swiglu)
    torch.cuda.synchronize()
    xd = xq.float() * xs[:, None]
    ref = xd @ w.dequant().t()
    if swiglu:
        g = (xd @ w.dequant().t()).reshape(M, -1, 2, 8)
        ref = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, -1)
    _check(out, ref, tol=3e-2)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("aligned", [True, False])
def test_gemm_mfma32_variant(fp8, swiglu, aligned):
    """The 32x32-MFMA tile variant (group_m bit 8; measured slower for bf16, not the default --
    profiles/r3_gemm_mfma32_experiment.jsonl) against fp32, ragged M and an N % 32 == 16 tail."""
    M, N, K = 777, 1040 if not swiglu else 1056, 1024
    x = _rand(M, K, seed=10, scale=0.5, offset=0.02)
    wb = _rand(N, K, seed=11, scale=0.03, offset=0.001)
    n_out = N // 2 if swiglu else N
    big = torch.zeros(M, n_out + 8, dtype=torch.bfloat16, device=DEV)
    out = big[:, :n_out] if aligned else big[:, 4:4 + n_out]
    if fp8:
        w = Fp8Weight.quantize(wb)
        xq, xs = hip.quant_fp8_rows(x)
        hip.gemm_fp8(xq, xs, w, out=out, swiglu=swiglu, group_m=4 | 256)
        y = (xq.float() * xs[:, None]) @ w.dequant().t()
    else:
        hip.gemm(x, wb, out=out, swiglu=swiglu, group_m=4 | 256)
        y = x.float() @ wb.float().t()
    torch.cuda.synchronize()
    if swiglu:
        g = y.reshape(M, -1, 2, 8)
        y = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, -1)
    _check(out, y, tol=3e-2)


def test_gemm_graph_capture():
    x, w = _rand(512, 1024, seed=10), _rand(768, 1024, seed=11, scale=0.05)
    out = torch.empty(512, 768, dtype=torch.bfloat16, device=DEV)
    hip.gemm(x, w, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        hip.gemm(x, w, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    _check(out, x.float() @ w.float().t())
