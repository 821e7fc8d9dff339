"""Engine on the CPU (reference ops): scheduling, KV paging, sampling rules."""

import math

import pytest
import torch

from llm_map_reduce_summarizer_amd.engine.chat import render_chat
from llm_map_reduce_summarizer_amd.engine.config import get_model_config
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
from llm_map_reduce_summarizer_amd.engine.kv_cache import PageAllocator
from llm_map_reduce_summarizer_amd.engine.tokenizer import get_tokenizer
from llm_map_reduce_summarizer_amd.ops import reference


@pytest.fixture(scope="module")
def eng():
    return LLMEngine(get_model_config("tiny", init_std=0.05), device="cpu", max_model_len=512, max_num_seqs=8,
                     kv_pages=64, sync_every=3, max_prefill_tokens=128)


def _prompts(k=5):
    return [[128000] + [(i * 31 + j * 7) % 100000 + 3 for j in range(8 + 23 * i)] for i in range(k)]


def test_lengths_and_pages_returned(eng):
    ps = [SamplingParams(1 + 3 * i, 0.3, i) for i in range(5)]
    outs = eng.generate(_prompts(), ps)
    assert [len(o.token_ids) for o in outs] == [p.max_new_tokens for p in ps]
    assert all(o.finish_reason == "length" for o in outs)
    assert eng.kv.alloc.available() == eng.kv.num_pages - 1
    assert [o.prompt_len for o in outs] == [len(p) for p in _prompts()]


def test_deterministic_and_batch_invariant(eng):
    ps = [SamplingParams(6, 0.3, 10 + i) for i in range(5)]
    a = eng.generate(_prompts(), ps)
    b = eng.generate(_prompts()[::-1], ps[::-1])[::-1]
    assert [o.token_ids for o in a] == [o.token_ids for o in b]


def test_greedy_decode_matches_full_prefill(eng):
    outs = eng.generate(_prompts(3), [SamplingParams(6, 0.0, 0)] * 3)
    for p, o in zip(_prompts(3), outs):
        nxt = eng.generate([p + o.token_ids[:-1]], [SamplingParams(1, 0.0, 0)])[0].token_ids[0]
        assert nxt == o.token_ids[-1]


def test_more_requests_than_slots_and_pages():
    eng = LLMEngine(get_model_config("tiny"), device="cpu", max_model_len=256, max_num_seqs=3, kv_pages=5,
                    page_size=64, sync_every=2)
    prompts = [[128000] + [i + j for j in range(30)] for i in range(7)]
    outs = eng.generate(prompts, [SamplingParams(4, 0.3, i) for i in range(7)])
    assert all(len(o.token_ids) == 4 for o in outs)
    assert eng.stats["peak_active"] <= 3


def test_eos_stops(eng):
    # force EOS: find the greedy first token of a prompt and declare it EOS
    p = _prompts(1)
    first = eng.generate(p, [SamplingParams(1, 0.0, 0)])[0].token_ids[0]
    eos_backup = list(eng.state.eos_ids)
    eng.state.set_eos([first])
    try:
        o = eng.generate(p, [SamplingParams(10, 0.0, 0)])[0]
        pinned = eng.generate(p, [SamplingParams(10, 0.0, 0)], ignore_eos=True)[0]
        assert eng.state.eos_ids == [first]  # restored after the ignore_eos call
    finally:
        eng.state.set_eos(eos_backup)
    assert o.token_ids == [first] and o.finish_reason == "stop"
    assert len(pinned.token_ids) == 10 and pinned.finish_reason == "length"


def test_rejects_bad_requests(eng):
    with pytest.raises(ValueError):
        eng.generate([[1] * 600], [SamplingParams(4)])
    with pytest.raises(ValueError):
        eng.generate([[200000]], [SamplingParams(4)])
    with pytest.raises(ValueError):
        eng.generate([[]], [SamplingParams(4)])


@pytest.mark.parametrize("native", [True, False])
def test_page_allocator(native):
    a = PageAllocator(10)
    if not native and a.native:
        a = PageAllocator.__new__(PageAllocator)
        a.num_pages, a._lib, a._h, a._free = 10, None, None, list(range(9, 0, -1))
    assert a.available() == 9
    x = a.alloc(4)
    assert 0 not in x and len(set(x)) == 4
    with pytest.raises(MemoryError):
        a.alloc(6)
    a.free(x)
    assert a.available() == 9
    assert a.alloc(1) == [x[0]]  # LIFO reuse


def test_native_allocator_double_free():
    a = PageAllocator(6)
    if not a.native:
        pytest.skip("runtime library not built")
    x = a.alloc(2)
    a.free(x)
    with pytest.raises(ValueError):
        a.free(x)
    with pytest.raises(ValueError):
        a.free([0])


def test_chat_template():
    tok = get_tokenizer()
    ids = render_chat(tok, "hello", "be brief")
    assert ids[0] == 128000 and ids.count(128009) == 2 and ids[-1] != 128009
    assert tok.decode(ids) .count("hello") == 1
    assert render_chat(tok, "hi")[1] == 128006


def test_decode_reference_matches_prefill_reference():
    torch.manual_seed(0)
    hq, hkv, d, page = 4, 2, 128, 16
    n = 37
    qkv = torch.randn(n, (hq + 2 * hkv) * d).to(torch.bfloat16)
    cu = torch.tensor([0, n], dtype=torch.int32)
    full = reference.attn_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d))
    kc = torch.zeros(8, hkv, page, d, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    bt = torch.tensor([[5, 2, 7, 1]], dtype=torch.int32)
    pos = torch.arange(n, dtype=torch.int32)
    reference.rope_kv(qkv.clone(), pos, torch.zeros(n, dtype=torch.int32), bt, kc, vc,
                      reference.rope_cos_sin(64, d, 1e4), hq, hkv, d, page)
    # the same K/V rotated (prefill path uses rotated qkv): rebuild and compare last row
    q2 = qkv.clone()
    reference.rope_kv(q2, pos, torch.zeros(n, dtype=torch.int32), bt, kc, vc, reference.rope_cos_sin(64, d, 1e4),
                      hq, hkv, d, page)
    full = reference.attn_prefill(q2, cu, hq, hkv, d, 1 / math.sqrt(d))
    last = reference.attn_decode(q2[n - 1:n], kc, vc, bt, torch.tensor([n - 1], dtype=torch.int32), hq, hkv, d,
                                 page, 1 / math.sqrt(d))
    assert torch.allclose(last.float(), full[n - 1:n].float(), atol=2e-2)


def test_gumbel_sampling_statistics():
    # Gumbel-max at temperature t samples softmax(logits / t)
    logits = torch.tensor([[1.0, 0.0, -1.0, 0.5]]).to(torch.bfloat16)
    counts = torch.zeros(4)
    for s in range(2000):
        tok = reference.sample_tokens(logits, torch.tensor([1.0]), torch.tensor([s]), torch.tensor([3]))
        counts[int(tok)] += 1
    p = torch.softmax(logits.float()[0], 0)
    assert torch.allclose(counts / counts.sum(), p, atol=0.04)


def test_fp8_weights_engine_cpu():
    cfg = get_model_config("tiny", init_std=0.05)
    e8 = LLMEngine(cfg, device="cpu", max_model_len=256, max_num_seqs=4, kv_pages=32, weight_dtype="fp8")
    e16 = LLMEngine(cfg, device="cpu", max_model_len=256, max_num_seqs=4, kv_pages=32)
    assert e8.model.weight_bytes() < e16.model.weight_bytes()  # embedding + head (bf16) dominate tiny
    p = [[128000] + list(range(50, 90))]
    o8 = e8.generate(p, [SamplingParams(4, 0.0, 0)])[0]
    assert len(o8.token_ids) == 4
    from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight
    w = torch.randn(64, 128)
    q = Fp8Weight.quantize(w)
    assert q.q.dtype == torch.float8_e4m3fn and torch.allclose(q.dequant(), w, rtol=0.07, atol=1e-3)


def test_prefill_export_import_roundtrip():
    """Disaggregated prefill: engine A prefills + exports (1 group), engine B imports the KV and first
    token and decodes -- same tokens as B generating on its own (same seeded weights)."""
    from llm_map_reduce_summarizer_amd.engine.engine import ImportedPrefill
    cfg = get_model_config("tiny", init_std=0.05)
    a = LLMEngine(cfg, device="cpu", max_model_len=512, max_num_seqs=8, kv_pages=64, sync_every=3)
    b = LLMEngine(cfg, device="cpu", max_model_len=512, max_num_seqs=8, kv_pages=64, sync_every=3)
    prompts = _prompts(4)
    ps = [SamplingParams(5 + i, 0.3, 40 + i) for i in range(4)]
    firsts, packs = a.prefill_export(prompts, ps, groups=1)
    assert a.kv.alloc.available() == a.kv.num_pages - 1  # exporter's pages released
    imported, off = {}, 0
    for i, p in enumerate(prompts):
        shape = b.import_shape(len(p))
        n = math.prod(shape)
        imported[i] = ImportedPrefill(firsts[i], packs[0][off:off + n].view(shape))
        off += n
    assert off == packs[0].numel()
    got = b.generate(prompts, ps, imported=imported)
    ref = b.generate(prompts, ps)
    assert [o.token_ids for o in got] == [o.token_ids for o in ref]
    assert b.stats["imported_prefills"] == 4
    # a request that is complete after its first token never reaches the decode loop
    one = b.generate(prompts[:1], [SamplingParams(1, 0.3, 40)], imported={0: ImportedPrefill(firsts[0], None)})
    assert one[0].token_ids == [firsts[0]] and one[0].finish_reason == "length"


def test_prefill_oom_is_isolated(monkeypatch):
    """A device OOM in a packed prefill is retried as halves (down to one sequence) with the same
    results; a single sequence that still does not fit re-raises."""
    e = LLMEngine(get_model_config("tiny", init_std=0.05), device="cpu", max_model_len=512, max_num_seqs=8,
                  kv_pages=64, sync_every=3, max_prefill_tokens=4096)
    ps = [SamplingParams(4, 0.3, 20 + i) for i in range(5)]
    ref = e.generate(_prompts(), ps)
    real = e._prefill
    calls = []

    def flaky(seqs):
        calls.append(len(seqs))
        if len(seqs) > 2:
            raise torch.OutOfMemoryError("simulated HIP out of memory")
        return real(seqs)

    monkeypatch.setattr(e, "_prefill", flaky)
    got = e.generate(_prompts(), ps)
    assert [o.token_ids for o in got] == [o.token_ids for o in ref]
    assert calls[:3] == [5, 2, 3] and e.stats["prefill_oom_splits"] == 2  # 5 -> 2 + 3 -> 2 + (1 + 2)
    assert e.kv.alloc.available() == e.kv.num_pages - 1

    def always(seqs):
        raise torch.OutOfMemoryError("simulated HIP out of memory")

    monkeypatch.setattr(e, "_prefill", always)
    with pytest.raises(torch.OutOfMemoryError):
        e.generate(_prompts(1), ps[:1])


def test_interleaved_prefill_oom_is_isolated(monkeypatch):
    """Requests joining a RUNNING batch (interleaved prefill): a device OOM in a packed slice pass re-runs
    the pass with half as many slices, down to one -- same tokens as without the fault, the running
    sequence keeps decoding, and a single slice that still does not fit re-raises."""
    def run(e):
        fed = []

        def feeder(done):
            if fed:
                return []
            fed.append(1)
            return [(p, SamplingParams(5, 0.3, 60 + i)) for i, p in enumerate(_prompts(4))]
        return e.generate(_prompts(1), [SamplingParams(12, 0.3, 59)], feeder=feeder)

    mk = lambda: LLMEngine(get_model_config("tiny", init_std=0.05), device="cpu", max_model_len=512,  # noqa: E731
                           max_num_seqs=8, kv_pages=64, sync_every=3, max_prefill_tokens=4096)
    ref = run(mk())
    e = mk()
    assert e.interleave
    real = e.model.prefill
    sizes = []

    def flaky(ids, positions, seq_idx, cu, last, tables, *a, **kw):
        if tables is e.pf_tables:
            sizes.append(len(kw["seqlens"]))
            if len(kw["seqlens"]) > 1:
                raise torch.OutOfMemoryError("simulated HIP out of memory")
        return real(ids, positions, seq_idx, cu, last, tables, *a, **kw)

    monkeypatch.setattr(e.model, "prefill", flaky)
    got = run(e)
    assert [o.token_ids for o in got] == [o.token_ids for o in ref]
    assert sizes[:3] == [4, 2, 1] and e.stats["prefill_oom_splits"] >= 2
    assert e.stats.get("interleaved_prefills", 0) == 4
    assert e.kv.alloc.available() == e.kv.num_pages - 1

    def always(ids, positions, seq_idx, cu, last, tables, *a, **kw):
        if tables is e.pf_tables:
            raise torch.OutOfMemoryError("simulated HIP out of memory")
        return real(ids, positions, seq_idx, cu, last, tables, *a, **kw)

    monkeypatch.setattr(e.model, "prefill", always)
    with pytest.raises(torch.OutOfMemoryError):
        run(e)


@pytest.mark.parametrize("chunk", [64, 192])
def test_chunked_prefill_equals_one_pass(chunk):
    """Prompts cut into end-aligned slices that attend to their cached prefix through the paged cache
    (ops.attn_prefill paged path) generate exactly what one-pass prefill generates (greedy, fp32 CPU)."""
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    prompts = [[128000] + [(i * 31 + j * 7) % 9000 + 5 for j in range(n)] for i, n in enumerate((450, 130, 61, 300))]
    sp = [SamplingParams(6, 0.0, i) for i in range(len(prompts))]
    outs = {}
    for c in (0, chunk):
        eng = LLMEngine(cfg, device="cpu", dtype=torch.float32, max_model_len=1024, max_num_seqs=8, kv_pages=96,
                        sync_every=3, prefill_chunk=c)
        outs[c] = [o.token_ids for o in eng.generate(prompts, sp)]
        if c:
            assert eng.stats["prefill_slices"] > len(prompts)
    assert outs[0] == outs[chunk]


def test_feeder_requests_join_the_running_batch(eng):
    """Streaming hook: requests returned by ``feeder`` join the running batch (no second generate) and
    produce exactly what a separate generate would (per-request seeds, batch-invariant engine)."""
    ps = [SamplingParams(4 + 5 * i, 0.3, 20 + i) for i in range(3)]
    extra = [SamplingParams(5, 0.3, 40 + i) for i in range(2)]
    seen = []

    def feeder(done):
        new = []
        for rid, o in done:
            seen.append(rid)
            if rid < 2:  # a follow-up for each of the first two requests, built from its output
                new.append(([128000] + o.token_ids, extra[rid]))
        return new

    calls = eng.stats["generate_calls"]
    outs = eng.generate(_prompts(3), ps, feeder=feeder)
    assert eng.stats["generate_calls"] == calls + 1 and len(outs) == 5
    assert sorted(seen) == [0, 1, 2, 3, 4] and seen.index(0) < seen.index(3)
    solo = eng.generate(_prompts(3), ps)
    assert [o.token_ids for o in outs[:3]] == [o.token_ids for o in solo]
    for k in range(2):
        ref = eng.generate([[128000] + solo[k].token_ids], [extra[k]])[0]
        assert outs[3 + k].token_ids == ref.token_ids and outs[3 + k].prompt_len == 1 + len(solo[k].token_ids)
    assert eng.kv.alloc.available() == eng.kv.num_pages - 1


def test_joining_prompt_prefills_between_decode_windows():
    """A long prompt that joins a RUNNING batch (feeder) is prefilled one slice per decode window: the
    running sequences keep producing tokens while it prefills (instead of stalling for its whole
    prefill), and every request generates exactly what the blocking admission generates."""
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    running = [[128000] + [(i * 31 + j * 7) % 9000 + 5 for j in range(40 + 9 * i)] for i in range(3)]
    joiner = [128000] + [(j * 13) % 9000 + 7 for j in range(600)]
    sp = [SamplingParams(40, 0.3, 70 + i) for i in range(3)]
    res = {}
    for inter in (True, False):
        eng = LLMEngine(cfg, device="cpu", dtype=torch.float32, max_model_len=1024, max_num_seqs=8, kv_pages=64,
                        sync_every=2, prefill_chunk=64)
        eng.interleave = inter
        fed, syncs = [], []

        def feeder(done, fed=fed):
            if not fed:
                fed.append(1)
                return [(joiner, SamplingParams(12, 0.3, 99))]
            return []

        def on_sync(tok_map, syncs=syncs):
            syncs.append(3 in tok_map)
        outs = eng.generate(running, sp, feeder=feeder, on_sync=on_sync)
        res[inter] = ([o.token_ids for o in outs], syncs, dict(eng.stats))
    assert res[True][0] == res[False][0]  # identical tokens, running and joined requests alike
    # windows the running rows decoded while the joiner was still prefilling: one per slice but its last
    before_join = lambda syncs: syncs.index(True)  # noqa: E731
    n_slices = -(-len(joiner) // 64)
    assert before_join(res[True][1]) - before_join(res[False][1]) >= n_slices - 1
    assert res[True][2]["interleaved_prefills"] == 1 and res[False][2].get("interleaved_prefills", 0) == 0
    assert res[True][2]["prefill_slices"] >= n_slices


def test_fp8_kv_cache_cpu():
    """The fp8 slab cache on the CPU reference path: rows round-trip within e4m3 precision, the layout sizes
    pages at ~1.94x per byte, and an fp8-KV engine's prefill logits stay close to the bf16-KV engine's."""
    from llm_map_reduce_summarizer_amd.engine.kv_cache import PagedKVCache
    from llm_map_reduce_summarizer_amd.ops import reference as R
    x = torch.randn(9, 2, 128) * 5
    x[3] = 0.0
    q, sc = R.kv8_quant_rows(x)
    assert torch.all(torch.log2(sc) == torch.round(torch.log2(sc)))  # powers of two
    deq = q.view(torch.float8_e4m3fn).float() * sc[..., None]
    assert float((deq - x).norm() / x.norm()) < 0.04 and float(deq[3].abs().sum()) == 0.0
    assert float(((x.abs().amax(-1) / sc)[torch.arange(9) != 3]).max()) <= 448.0
    # rows far below e4m3's range (max|x| < 448 * 2^-126): the scale stays a normal 2^-126, so 1 / scale is
    # finite and the row quantises to finite bytes (zero elements stay zero) -- never NaN
    tiny = torch.zeros(3, 128)
    tiny[0, 5] = 1e-36
    tiny[1, :] = 3e-37
    tiny[2, 7] = -2e-37
    qt, st = R.kv8_quant_rows(tiny)
    assert torch.all(st == 2.0 ** -126) and torch.all(torch.isfinite(1.0 / st))
    dq = qt.view(torch.float8_e4m3fn).float()
    assert torch.all(torch.isfinite(dq)) and float(dq[0, :5].abs().sum()) == 0.0
    b = PagedKVCache.size_pages(1 << 30, 32, 8, 64, 128)
    f = PagedKVCache.size_pages(1 << 30, 32, 8, 64, 128, kv_dtype="fp8")
    assert 1.9 < f / b < 2.0
    fv = PagedKVCache.size_pages(1 << 30, 32, 8, 64, 128, kv_dtype="fp8v")
    assert 1.3 < fv / b < 1.35  # bf16 K + fp8 V: 24.25 of 32 KiB per (page, head)
    prompts = [[128000] + [(i * 37 + j * 11) % 120000 + 5 for j in range(n)] for i, n in enumerate((300, 129))]
    rec = {}
    for kvd in ("bf16", "fp8", "fp8v"):
        e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cpu", max_model_len=1024,
                      max_num_seqs=4, kv_pages=32, kv_dtype=kvd, prefill_chunk=128)
        r = []
        orig = e._sample
        e._sample = lambda lg, v, r=r, orig=orig: (r.append(lg.float().clone()), orig(lg, v))
        e.generate(prompts, [SamplingParams(1, 0.0, 0)] * 2)
        rec[kvd] = r[-1]
    a, b = rec["bf16"], rec["fp8"]
    assert float((a - b).norm() / a.norm()) < 0.15
    e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cpu", max_model_len=1024,
                  max_num_seqs=4, kv_pages=32, kv_dtype="fp8v", prefill_chunk=128)
    assert e.kv.k.dtype == torch.bfloat16 and e.kv.v.dtype == torch.uint8 and e.kv.fp8
    # V-only rounding: closer to bf16 KV than the K+V variant
    assert float((a - rec["fp8v"]).norm() / a.norm()) <= float((a - b).norm() / a.norm()) + 1e-6


def test_pinned_windows_run_to_the_first_length_stop():
    """ignore_eos: no row can stop before its max_new_tokens, so the host syncs only when the first row runs
    out of steps (LLMEngine._window), not every sync_every steps -- with identical tokens."""
    cfg = get_model_config("tiny", init_std=0.05)
    ps = [SamplingParams(5 + 4 * i, 0.3, 20 + i) for i in range(4)]
    outs, wins = [], []
    for se in (2, 64):
        e = LLMEngine(cfg, device="cpu", max_model_len=512, max_num_seqs=8, kv_pages=64, sync_every=se)
        outs.append([o.token_ids for o in e.generate(_prompts(4), ps, ignore_eos=True)])
        wins.append(e.stats["decode_windows"])
        assert e.state.eos_ids  # re-armed after the pinned call
        armed = e.generate(_prompts(4), ps)  # EOS armed: sync_every windows again
        assert [len(o.token_ids) for o in armed] <= [p.max_new_tokens for p in ps]
    assert outs[0] == outs[1]
    assert [len(t) for t in outs[0]] == [p.max_new_tokens for p in ps]
    # max_new 5 / 9 / 13 / 17 (first token sampled at prefill): windows of 4, 4, 4, 4 steps at most
    assert wins[0] == wins[1] == 4


def test_window_rule():
    e = LLMEngine(get_model_config("tiny"), device="cpu", max_model_len=256, max_num_seqs=4, kv_pages=16,
                  sync_every=16)
    assert e._window([], False) == 0 and e._window([0, 0], False) == 0
    assert e._window([40, 7], False) == 16  # EOS armed: sync_every, bounded by the longest row
    assert e._window([5, 3], False) == 5
    e.state.set_eos([])
    assert e._window([40, 7], False) == 7  # pinned: until the first row runs out
    assert e._window([4000, 3000], False) == 256  # at most MAX_WINDOW
    assert e._window([40, 7], True) == 16  # a feeder / stream hook / interleaved prefill wants sync points
