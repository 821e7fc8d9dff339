"""Engine-level GPU tests: decode path consistent with a full prefill,
hipGraph replay identical to eager, batching-invariant sampling."""

import pytest
import torch

pytestmark = pytest.mark.gpu

from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams  # noqa: E402


@pytest.fixture(scope="module")
def eng():
    return LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cuda:0", max_model_len=2048,
                     max_num_seqs=16, kv_pages=256, sync_every=8)


def _prompts():
    return [[128000] + [(i * 37 + j * 11) % 120000 + 5 for j in range(n)] for i, n in enumerate((40, 300, 7, 129))]


def test_native_kernels_loaded(eng):
    eng.generate([[128000, 5, 6, 7]], [SamplingParams(2, 0.0, 0)])
    maps = open("/proc/self/maps").read()
    assert "libmrsum_kernels.so" in maps


def test_greedy_decode_matches_prefill(eng):
    prompts = _prompts()
    outs = eng.generate(prompts, [SamplingParams(12, 0.0, 0)] * len(prompts))
    # teacher-forced: prefill prompt + generated[:k] -> next greedy token must be generated[k]
    agree = 0
    for p, o in zip(prompts, outs):
        full = p + o.token_ids[:-1]
        check = eng.generate([full], [SamplingParams(1, 0.0, 0)])[0].token_ids[0]
        agree += check == o.token_ids[-1]
    assert agree >= len(prompts) - 1  # a bf16 near-tie may flip one argmax


def test_graph_equals_eager(eng):
    prompts = _prompts()
    sp = [SamplingParams(10, 0.3, 5 + i) for i in range(len(prompts))]
    a = eng.generate(prompts, sp)
    eng.use_graphs = False
    try:
        b = eng.generate(prompts, sp)
    finally:
        eng.use_graphs = True
    assert [o.token_ids for o in a] == [o.token_ids for o in b]


def test_order_invariance(eng):
    """Per-request seeds + row-independent kernels: permuting the batch permutes the outputs."""
    prompts = _prompts()
    sp = [SamplingParams(10, 0.3, 100 + i) for i in range(len(prompts))]
    a = eng.generate(prompts, sp)
    b = eng.generate(prompts[::-1], sp[::-1])[::-1]
    same = sum(x.token_ids == y.token_ids for x, y in zip(a, b))
    assert same >= len(prompts) - 1


def test_many_sequences_compaction(eng):
    prompts = [[128000] + [(i * 13 + j) % 5000 + 10 for j in range(20 + 7 * i)] for i in range(12)]
    sp = [SamplingParams(3 + (i % 5) * 4, 0.3, i) for i in range(12)]
    outs = eng.generate(prompts, sp)
    assert [len(o.token_ids) for o in outs] == [s.max_new_tokens for s in sp]
    assert eng.kv.alloc.available() == eng.kv.num_pages - 1


def test_packed_prefill_matches_single(eng):
    """A packed varlen prefill of ragged prompts (3803 rows: no 256-multiple, no padding) generates what
    each prompt generates on its own."""
    prompts = [[128000] + [(i * 53 + j * 7) % 120000 + 5 for j in range(n)] for i, n in enumerate((1500, 1200, 1100))]
    sp = [SamplingParams(8, 0.0, 0)] * len(prompts)
    a = eng.generate(prompts, sp)
    b = [eng.generate([p], [s])[0] for p, s in zip(prompts, sp)]
    same = sum(x.token_ids == y.token_ids for x, y in zip(a, b))
    assert same >= len(prompts) - 1  # a bf16 near-tie may flip one sequence


def test_chunked_prefill_matches_one_pass():
    """Chunked prefill (end-aligned slices through the paged cache) generates what one-pass prefill does
    (greedy; a bf16 near-tie may flip one sequence)."""
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    prompts = [[128000] + [(i * 53 + j * 7) % 120000 + 5 for j in range(n)] for i, n in enumerate((1500, 700, 2600, 90))]
    sp = [SamplingParams(8, 0.0, 0)] * len(prompts)
    res = {}
    for c in (0, 512):
        e = LLMEngine(cfg, device="cuda:0", max_model_len=4096, max_num_seqs=8, kv_pages=256, sync_every=8,
                      prefill_chunk=c)
        res[c] = [o.token_ids for o in e.generate(prompts, sp)]
        if c:
            assert e.stats["prefill_slices"] > len(prompts)
    same = sum(a == b for a, b in zip(res[0], res[512]))
    assert same >= len(prompts) - 1, (res[0], res[512])


def test_long_context_class_graphs():
    """Prompts in the 6k-12k and 12k-32k context classes run on their own decode graphs (attention split
    plans per class) and agree with teacher-forced prefill, like the short class."""
    e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05, max_position=40960), device="cuda:0",
                  max_model_len=40960, max_num_seqs=4, kv_pages=1400, sync_every=8)
    for n in (7000, 20000):
        p = [128000] + [(j * 29 + n) % 120000 + 5 for j in range(n)]
        out = e.generate([p], [SamplingParams(6, 0.0, 0)])[0]
        assert (1, 1 if n < 12288 else 2) in e._graphs
        nxt = e.generate([p + out.token_ids[:-1]], [SamplingParams(1, 0.0, 0)])[0].token_ids[0]
        assert nxt == out.token_ids[-1]


def test_fp8_engine_decode_matches_prefill():
    """fp8 (e4m3fn) weights: decode GEMMs on the fp8 stream / register-streaming kernels, prefill on
    the fp8 MFMA GEMM (gemm.hip) -- greedy decode agrees with teacher-forced prefill."""
    e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cuda:0", max_model_len=2048,
                  max_num_seqs=16, kv_pages=256, sync_every=8, weight_dtype="fp8")
    prompts = _prompts()
    outs = e.generate(prompts, [SamplingParams(8, 0.0, 0)] * len(prompts))
    agree = 0
    for p, o in zip(prompts, outs):
        nxt = e.generate([p + o.token_ids[:-1]], [SamplingParams(1, 0.0, 0)])[0].token_ids[0]
        agree += nxt == o.token_ids[-1]
    assert agree >= len(prompts) - 1


def test_feeder_follow_up_joins_running_batch_across_context_class():
    """Streaming hook on the GPU engine: a fed follow-up whose context crosses into the 6k-12k class
    joins the running batch (the decode graphs switch class mid-generate) and generates what a
    separate generate does."""
    e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05, max_position=16384), device="cuda:0",
                  max_model_len=16384, max_num_seqs=8, kv_pages=1400, sync_every=4)
    prompts = [[128000] + [(i * 41 + j * 3) % 120000 + 5 for j in range(n)] for i, n in enumerate((60, 300))]
    sp = [SamplingParams(4, 0.0, 0), SamplingParams(24, 0.0, 0)]
    long_p = [128000] + [(j * 17) % 120000 + 5 for j in range(6900)]

    def feeder(done):
        return [(long_p + o.token_ids, SamplingParams(6, 0.0, 0)) for rid, o in done if rid == 0]

    outs = e.generate(prompts, sp, feeder=feeder)
    assert len(outs) == 3 and e.stats.get("fed_requests") == 1 and e._ctx_cls == 1
    ref = e.generate([long_p + outs[0].token_ids], [SamplingParams(6, 0.0, 0)])[0]
    assert outs[2].token_ids == ref.token_ids
    assert outs[1].token_ids == e.generate([prompts[1]], [sp[1]])[0].token_ids


def test_streamed_map_reduce_pipeline_on_gpu():
    """The streamed map -> level-1 reduce (engine feeder, decode graphs across batch buckets) end to end on
    the GPU engine: level 1 runs inside the map's generate call and the run completes with a summary."""
    import asyncio

    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.pipeline.executor import LLMExecutor
    from llm_map_reduce_summarizer_amd.pipeline.orchestrator import TranscriptSummarizer
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    cfg = LLMConfig(MAX_TOKENS=12)
    prov = LocalEngineProvider("tiny-gqa4", cfg, device="cuda:0", max_model_len=4096, ignore_eos=True,
                               engine_options={"kv_pages": 512, "max_num_seqs": 16})
    ex = LLMExecutor(config=cfg, provider_obj=prov)
    summ = TranscriptSummarizer(executor=ex, max_tokens_per_chunk=1000, stream_reduce=True,
                                aggregator_options={"max_tokens_per_batch": 60})
    rep = asyncio.run(summ.summarize(synthetic_transcript(0.5, seed=3)))
    st = prov.stats()
    assert rep["reduce_plan"].get("level1_streamed") and rep["reduce_plan"]["calls"][0] >= 2
    assert st.get("fed_requests", 0) == rep["reduce_plan"]["calls"][0] and st["generate_calls"] == 2
    assert rep["summary"] and rep["failed_chunks"] == 0


def test_32k_prompt_joins_running_batch_interleaved():
    """A 32k-token prompt joining a running 15-sequence batch (feeder) is prefilled one 4096-token slice
    per decode window: the running sequences' longest pause between two decode windows stays within
    1.5x one slice's forward time (not the whole 32k prefill), and every request generates exactly the
    tokens of the blocking admission (same 16-row bucket before and after the join: row-independent
    kernels).  Llama-3-8B layer shapes, 4 layers."""
    cfg = get_model_config("llama3.1-8b", n_layers=4)
    running = [[128000] + [(i * 37 + j * 11) % 120000 + 5 for j in range(1500 + 50 * i)] for i in range(15)]
    joiner = [128000] + [(j * 13) % 120000 + 7 for j in range(32000)]
    sp = [SamplingParams(240, 0.3, 70 + i) for i in range(15)]
    res = {}
    for inter in (True, False):
        e = LLMEngine(cfg, device="cuda:0", max_model_len=33 * 1024, max_num_seqs=16, kv_fraction=0.3,
                      sync_every=8, prefill_chunk=4096)
        e.interleave = inter
        e.generate(running[:2], sp[:2])  # warm: graphs / kernel loads outside the measured run
        e.stats["max_window_gap_s"] = 0.0
        fed = []

        def feeder(done, fed=fed):
            if not fed:
                fed.append(1)
                return [(joiner, SamplingParams(16, 0.3, 99))]
            return []
        outs = e.generate(running, sp, feeder=feeder)
        res[inter] = ([o.token_ids for o in outs], dict(e.stats))
        del e
        torch.cuda.empty_cache()
    toks_i, st_i = res[True]
    toks_b, st_b = res[False]
    assert toks_i == toks_b
    assert st_i["interleaved_prefills"] == 1
    slice_s = st_i["interleaved_pass_max_s"]
    assert st_i["max_window_gap_s"] <= 1.5 * slice_s, (st_i["max_window_gap_s"], slice_s)
    # the blocking admission stalled the running rows for the whole (8-slice) prefill
    assert st_b["max_window_gap_s"] > 4 * slice_s, (st_b["max_window_gap_s"], slice_s)


@pytest.mark.parametrize("capture_first", ["ignore", "honour"])
def test_eos_is_read_at_graph_replay(capture_first):
    """EOS handling must not depend on which generate captured the decode graphs (the stop ids are
    device state read by the sampler at every replay, sampler.hip EOS_SLOTS): a decode-produced greedy
    token declared EOS stops an EOS-honouring call and is ignored by an ignore_eos call, whichever of
    the two ran (and captured) first -- and after an explicit capture_graphs() at start-up."""
    def fresh():
        e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cuda:0", max_model_len=1024,
                      max_num_seqs=8, kv_pages=64, sync_every=4)
        e.state.set_eos([])
        return e

    prompt = [[128000] + [(j * 29) % 50000 + 11 for j in range(60)]]
    probe = fresh()
    probe.use_graphs = False
    ref = probe.generate(prompt, [SamplingParams(12, 0.0, 0)])[0].token_ids
    k = next((i for i in range(3, 12) if ref[i] not in ref[:i]), None)
    assert k is not None, "greedy sequence without a fresh decode-produced token"
    stop = ref[k]
    del probe
    for eager_capture in (False, True):
        eng = fresh()
        eng.state.set_eos([stop])
        if eager_capture:
            assert eng.capture_graphs(max_batch=1) >= 1
        calls = [("ignore", True), ("honour", False)]
        if capture_first == "honour":
            calls.reverse()
        for name, ign in calls:
            o = eng.generate(prompt, [SamplingParams(12, 0.0, 0)], ignore_eos=ign)[0]
            if ign:
                assert o.token_ids == ref and o.finish_reason == "length", (name, eager_capture)
            else:
                assert o.token_ids == ref[:k + 1] and o.finish_reason == "stop", (name, eager_capture)
        assert eng.state.eos_ids == [stop]
        assert eng.stats["graph_captures"] >= 1


def test_gqa_ratio3_model_runs():
    """A GQA 3:1 model (Llama-3.2-3B's ratio) prefills and decodes through the attention kernels'
    per-query-head fallback; greedy decode agrees with a teacher-forced prefill."""
    e = LLMEngine(get_model_config("tiny-gqa3", init_std=0.05), device="cuda:0", max_model_len=2048,
                  max_num_seqs=8, kv_pages=128, sync_every=4)
    prompts = _prompts()
    outs = e.generate(prompts, [SamplingParams(8, 0.0, 0)] * len(prompts))
    assert all(len(o.token_ids) == 8 for o in outs)
    agree = sum(e.generate([p + o.token_ids[:-1]], [SamplingParams(1, 0.0, 0)])[0].token_ids[0] == o.token_ids[-1]
                for p, o in zip(prompts, outs))
    assert agree >= len(prompts) - 1


@pytest.mark.parametrize("kvd", ["fp8v", "fp8"])
def test_fp8_kv_cache_engine(kvd):
    """fp8 slab caches (fp8v: V only, the --kv-dtype variant; fp8: K and V, an engine format not offered by the
    CLI): graph-replayed decode over the cache agrees with a teacher-forced prefill of the same engine
    (chunked through the cache)."""
    e = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cuda:0", max_model_len=2048,
                  max_num_seqs=8, kv_pages=128, sync_every=4, kv_dtype=kvd, prefill_chunk=128)
    assert e.kv.v.dtype == torch.uint8 and e.kv.v.shape[-1] == 64 * 128 + 4 * 64
    assert e.kv.k.dtype == (torch.uint8 if kvd == "fp8" else torch.bfloat16)
    prompts = _prompts()
    outs = e.generate(prompts, [SamplingParams(8, 0.0, 0)] * len(prompts))
    assert all(len(o.token_ids) == 8 for o in outs) and e.stats["graph_captures"] >= 1
    agree = sum(e.generate([p + o.token_ids[:-1]], [SamplingParams(1, 0.0, 0)])[0].token_ids[0] == o.token_ids[-1]
                for p, o in zip(prompts, outs))
    assert agree >= len(prompts) - 1


def test_pinned_windows_match_short_windows(eng, monkeypatch):
    """ignore_eos: one window of up to MAX_WINDOW graph replays per batch (LLMEngine._window) gives the same
    tokens as 2-step windows with a host sync between them (equal max_new: same batch composition)."""
    prompts = _prompts()
    ps = [SamplingParams(40, 0.3, 7 + i) for i in range(len(prompts))]
    w0 = eng.stats.get("decode_windows", 0)
    long_w = eng.generate(prompts, ps, ignore_eos=True)
    n_long = eng.stats["decode_windows"] - w0
    monkeypatch.setattr(LLMEngine, "_window", lambda self, left, hooked: min(2, max([0] + left)))
    w1 = eng.stats["decode_windows"]
    short_w = eng.generate(prompts, ps, ignore_eos=True)
    n_short = eng.stats["decode_windows"] - w1
    assert [o.token_ids for o in long_w] == [o.token_ids for o in short_w]
    assert all(len(o.token_ids) == 40 for o in long_w)
    assert n_long == 1 and n_short == 20  # 39 steps after the prefill's token: one window vs twenty
