"""Map executor, reduce aggregator, orchestrator and CLI on the mock provider
(BASELINE config 1: the reference example end-to-end on CPU, no GPU, no keys)."""

import asyncio
import json
import os

import pytest

from llm_map_reduce_summarizer_amd.config import LLMConfig
from llm_map_reduce_summarizer_amd.pipeline.aggregator import ResultAggregator
from llm_map_reduce_summarizer_amd.pipeline.executor import LLMExecutor
from llm_map_reduce_summarizer_amd.pipeline.orchestrator import TranscriptSummarizer
from llm_map_reduce_summarizer_amd.pipeline.prompts import render_template
from llm_map_reduce_summarizer_amd.pipeline.providers import GenRequest, GenResult, MockProvider, Provider


def _cfg(**kw):
    kw.setdefault("RETRY_DELAY", 0.0)
    return LLMConfig(**kw)


def _chunks(n):
    return [{"chunk_index": i, "start_time": 60.0 * i, "end_time": 60.0 * (i + 1),
             "text_with_context": "chunk %d text" % i, "text": "t"} for i in range(n)]


class EchoProvider(Provider):
    """Records requests; returns a long deterministic text to drive the reduce planner."""
    name = "echo"

    def __init__(self, words=400):
        super().__init__("echo")
        self.reqs = []
        self.words = words

    async def generate(self, req):
        self.reqs.append(req)
        return GenResult(" ".join(["word%d" % (i % 50) for i in range(self.words)]), 10, self.words)


def test_executor_schema_and_counters():
    ex = LLMExecutor(config=_cfg(), provider="mock")
    out = asyncio.run(ex.process_chunks(_chunks(4)[::-1], "Summarize: {transcript} ({summary_type})",
                                        system_prompt="sys"))
    assert [c["chunk_index"] for c in out] == [0, 1, 2, 3]
    for c in out:
        assert c["summary"].startswith("[Mock Mock Response") or c["summary"].startswith("[Mock")
        assert c["tokens_used"] == 100 and c["system_prompt"] == "sys" and "processing_index" in c
    assert ex.total_requests == 4 and ex.failed_requests == 0 and ex.total_tokens_used == 400


def test_executor_retries_then_error_summary():
    ex = LLMExecutor(config=_cfg(RETRY_ATTEMPTS=3), provider_obj=MockProvider(fault_rate=1.0))
    out = asyncio.run(ex.process_chunks(_chunks(2), "{transcript}"))
    assert all(c["summary"].startswith("[Error processing chunk: ") and "error" in c for c in out)
    assert ex.failed_requests == 2
    ex2 = LLMExecutor(config=_cfg(RETRY_ATTEMPTS=6), provider_obj=MockProvider(fault_rate=0.5, seed=3))
    out2 = asyncio.run(ex2.process_chunks(_chunks(8), "{transcript}"))
    assert sum(1 for c in out2 if "error" in c) <= 1  # transient faults are absorbed by retries


def test_prompt_braces_do_not_crash():
    # reference bug Q7: a stray {"a"} in a prompt file raised KeyError
    assert render_template('json: {"a": 1} {transcript} {{x}}', transcript="T") == 'json: {"a": 1} T {x}'


def test_aggregator_single_vs_hierarchical():
    prov = EchoProvider(words=30)
    ex = LLMExecutor(config=_cfg(), provider_obj=prov)
    agg = ResultAggregator(executor=ex)
    chunks = [dict(c, summary="short summary %d" % c["chunk_index"]) for c in _chunks(5)]
    r = asyncio.run(agg.aggregate(chunks, metadata={"File": "x"}))
    assert {k: r["plan"][k] for k in ("levels", "calls")} == {"levels": 1, "calls": [1]}
    assert r["chunks_aggregated"] == 5 and len(r["plan"]["seconds"]) == 1
    assert "[Time: 00:00 - 01:00]" in prov.reqs[-1].user and "File: x" in prov.reqs[-1].user
    assert prov.reqs[-1].temperature == pytest.approx(0.2)

    long = " ".join(["lorem%d ipsum" % i for i in range(450)])
    chunks = [dict(c, summary=long) for c in _chunks(23)]
    prov.reqs.clear()
    r = asyncio.run(agg.aggregate(chunks))
    n_tok = agg.tokenizer.count("[Time: 00:00 - 01:00]\n" + long)
    bs = min(10, max(1, int(5000 / n_tok)))
    assert r["plan"]["levels"] == 2 and r["plan"]["calls"] == [-(-23 // bs), 1]
    assert len(r["plan"]["seconds"]) == 2 and all(t >= 0 for t in r["plan"]["seconds"])
    assert "Batch: 1/%d" % r["plan"]["calls"][0] in prov.reqs[0].user


def test_aggregator_recursive_mode_and_custom_prompt():
    prov = EchoProvider(words=500)
    ex = LLMExecutor(config=_cfg(), provider_obj=prov)
    agg = ResultAggregator(executor=ex, max_levels=None)
    chunks = [dict(c, summary=" ".join(["w%d" % i for i in range(1200)])) for c in _chunks(30)]
    r = asyncio.run(agg.aggregate(chunks, prompt_template="TIMELINE SUMMARY\n{summaries}\nn={num_summaries}"))
    assert r["plan"]["levels"] >= 3
    assert prov.reqs[-1].user.startswith("TIMELINE SUMMARY") and "SUMMARY 1:" in prov.reqs[-1].user


def test_orchestrator_on_reference_example(example_transcript, tmp_path):
    s = TranscriptSummarizer(provider="mock", max_tokens_per_chunk=4000)
    save = tmp_path / "chunks.json"
    rep = asyncio.run(s.summarize(example_transcript, save_intermediate_chunks=str(save),
                                  metadata={"Speaker": "x"}))
    for k in ("summary", "processing_time", "tokens_used", "cost", "segments", "chunks", "provider", "model"):
        assert k in rep
    assert rep["segments"] == 4778 and rep["provider"] == "mock" and rep["chunks"] > 20
    data = json.loads(save.read_text())
    assert set(data) == {"timestamp", "chunks"} and len(data["chunks"]) == rep["chunks"]
    assert set(data["chunks"][0]) == {"chunk_index", "start_time", "end_time", "summary", "tokens_used"}
    # resume from the saved file skips the map stage
    rep2 = asyncio.run(TranscriptSummarizer(provider="mock").summarize(example_transcript,
                                                                        resume_chunks=str(save)))
    assert rep2["chunks"] == rep["chunks"] and rep2["tokens_used"] == 0


def test_cli_mock_end_to_end(example_transcript, tmp_path, capsys):
    from llm_map_reduce_summarizer_amd.cli import main
    inp = tmp_path / "t.json"
    inp.write_text(json.dumps({"segments": example_transcript["segments"][:600]}))
    out = tmp_path / "o" / "summary.md"
    rc = main(["-i", str(inp), "-o", str(out), "--provider", "mock", "--report", "-q",
               "--max-tokens-per-chunk", "2000"])
    assert rc == 0 and out.read_text().startswith("# Transcript Summary")
    rep = json.loads(out.with_suffix(".report.json").read_text())
    assert rep["provider"] == "mock" and rep["segments"] == 600
    assert main(["-i", str(tmp_path / "missing.json"), "--provider", "mock"]) == 1


def test_cli_profile_trace(example_transcript, tmp_path):
    from llm_map_reduce_summarizer_amd.cli import main
    inp = tmp_path / "t.json"
    inp.write_text(json.dumps({"segments": example_transcript["segments"][:50]}))
    prof = tmp_path / "prof"
    assert main(["-i", str(inp), "--provider", "mock", "-q", "--profile", str(prof)]) == 0
    trace = json.loads((prof / "trace_rank0.json").read_text())
    assert "traceEvents" in trace and (prof / "kernels_rank0.txt").exists()


def test_simple_aggregator_one_shot():
    from llm_map_reduce_summarizer_amd.pipeline.simple_aggregator import SimpleAggregator, aggregate_summaries
    prov = EchoProvider(words=5)
    ex = LLMExecutor(config=_cfg(), provider_obj=prov)
    out = asyncio.run(SimpleAggregator(executor=ex).aggregate(["a", "b"], {"File": "f"}))
    assert out.startswith("word0") and len(prov.reqs) == 1
    r = prov.reqs[0]
    assert "SUMMARY 2:" in r.user and "- File: f" in r.user and r.temperature == pytest.approx(0.2)
    assert r.system.strip().startswith("You are a professional transcript summarizer")
    ex2 = LLMExecutor(config=_cfg(RETRY_ATTEMPTS=1), provider_obj=MockProvider(fault_rate=1.0))
    assert aggregate_summaries(["x"], executor=ex2).startswith("Error generating summary: ")


class TimedProvider(Provider):
    """Per-request provider with a latency per chunk index; records (event, stage, tag, time)."""
    name = "timed"

    def __init__(self, fail_once=()):
        super().__init__("timed")
        self.events = []
        self.fail_once = set(fail_once)
        self.l1_users = []

    async def generate(self, req):
        import time as _t
        self.events.append(("start", req.stage, req.tag, _t.perf_counter()))
        if req.stage == "map":
            await asyncio.sleep(0.004 * (1 + req.tag))
            if req.tag in self.fail_once:
                self.fail_once.discard(req.tag)
                raise RuntimeError("flaky chunk %d" % req.tag)
            text = " ".join(["c%dw%d" % (req.tag, i) for i in range(300)])
        else:
            if req.stage == "reduce_l1":
                self.l1_users.append(req.user)
            text = "reduced " + req.stage
        self.events.append(("end", req.stage, req.tag, _t.perf_counter()))
        return GenResult(text, 10, 300)


def _stream_summarizer(prov, stream, **agg):
    ex = LLMExecutor(config=_cfg(MAX_TOKENS=300), provider_obj=prov)
    return TranscriptSummarizer(executor=ex, stream_reduce=stream, max_tokens_per_chunk=400,
                                aggregator_options=dict({"max_tokens_per_batch": 1500}, **agg))


def test_streamed_level1_starts_before_the_map_ends():
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    prov = TimedProvider()
    rep = asyncio.run(_stream_summarizer(prov, True).summarize(synthetic_transcript(1.0, seed=1)))
    plan = rep["reduce_plan"]
    assert plan.get("level1_streamed") and plan["levels"] == 2 and plan["calls"][0] >= 2
    first_l1 = min(t for ev, st, _, t in prov.events if ev == "start" and st == "reduce_l1")
    last_map = max(t for ev, st, _, t in prov.events if ev == "end" and st == "map")
    assert first_l1 < last_map  # no map -> reduce barrier
    assert rep["summary"] == "reduced reduce_final" and rep["failed_chunks"] == 0
    # every chunk appears in exactly one level-1 request, batches in transcript order
    for i in range(rep["chunks"]):
        assert sum(1 for u in prov.l1_users if "c%dw0 " % i in u) == 1


def test_streamed_level1_equals_barrier_with_the_same_batches():
    """Same batches => same level-1 prompts and the same final prompt as the barrier reduce."""
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    tr = synthetic_transcript(1.0, seed=2)
    ps, pb = TimedProvider(), TimedProvider()
    s_stream = _stream_summarizer(ps, True)
    rs = asyncio.run(s_stream.summarize(tr))
    bs = len(s_stream.aggregator.stream_plan([{"chunk_index": i} for i in range(rs["chunks"])])[0])
    s_bar = _stream_summarizer(pb, False)
    s_bar._ensure_components()
    s_bar.aggregator._calculate_batch_size = lambda cur: bs
    rb = asyncio.run(s_bar.summarize(tr))
    assert rs["reduce_plan"]["calls"] == rb["reduce_plan"]["calls"]
    assert sorted(ps.l1_users) == sorted(pb.l1_users)
    fin = lambda p: [e for e in p.events if e[1] == "reduce_final"]
    assert len(fin(ps)) == len(fin(pb)) == 2 and rs["summary"] == rb["summary"]


def test_streamed_retries_a_failed_chunk_before_its_batch():
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    prov = TimedProvider(fail_once={1})
    rep = asyncio.run(_stream_summarizer(prov, True).summarize(synthetic_transcript(1.0, seed=1)))
    assert rep["failed_chunks"] == 0
    assert sum(1 for u in prov.l1_users if "c1w0 " in u) == 1 and not any("Error" in u for u in prov.l1_users)


class BatchedGroupsProvider(Provider):
    """Batched provider with a streaming path that reports one chunk as failed in the streamed pass."""
    name = "bg"
    batched = True

    def __init__(self, bad=2, words=300):
        super().__init__("bg")
        self.bad = bad
        self.batches = []
        self.pad = " ".join("w%d" % i for i in range(words))  # summaries long enough for 2 levels

    async def generate_batch(self, reqs):
        self.batches.append([r.stage for r in reqs])
        return [GenResult("ok %s %s %s" % (r.stage, r.tag, self.pad), 5, 5) for r in reqs]

    async def generate_groups(self, reqs, groups, build):
        first = [GenResult("", error="boom") if i == self.bad else GenResult("s%d %s" % (i, self.pad), 5, 5)
                 for i in range(len(reqs))]
        second = []
        for g, members in enumerate(groups):
            r2 = build(g, [first[i] for i in members])
            second.append(None if r2 is None else GenResult("l1 %d" % g, 5, 5))
        self.batches.append(["streamed"])
        return first, second


def test_streamed_batched_failure_reruns_only_the_affected_batch():
    prov = BatchedGroupsProvider(bad=2)
    ex = LLMExecutor(config=_cfg(MAX_TOKENS=300), provider_obj=prov)
    agg = ResultAggregator(executor=ex, max_tokens_per_batch=1500)
    chunks = _chunks(9)
    groups = agg.stream_plan(chunks)
    assert groups and all(len(g) == len(groups[0]) for g in groups[:-1])
    n = len(groups)
    recs, l1 = asyncio.run(ex.process_chunks_streamed(chunks, "{transcript}", groups,
                                                      lambda g, rs: agg.level1_request(g, n, rs)))
    assert recs[2]["summary"].startswith("ok map 2") and "error" not in recs[2]  # retried via generate_batch
    gbad = next(g for g, m in enumerate(groups) if 2 in m)
    assert l1[gbad] is None and all(l1[g] is not None for g in range(n) if g != gbad)
    # the dropped follow-up of the failed group is not counted: the aggregator re-runs (and counts) it
    assert ex.failed_requests == 0 and ex.total_requests == 9 + n - 1
    r = asyncio.run(agg.aggregate(recs, level1=(groups, l1)))
    assert r["plan"]["calls"] == [n, 1] and r["plan"]["level1_streamed"]
    assert prov.batches[-2] == ["reduce_l1"] and prov.batches[-1] == ["reduce_final"]
    assert ex.total_requests == 9 + n + 1  # every request counted exactly once


def test_streamed_level1_short_summaries_reduce_in_one_pass():
    """Streamed groups are planned for summaries at the token cap; when the real ones fit one reduce
    call, the reference's single pass runs (no extra level)."""
    prov = BatchedGroupsProvider(bad=-1, words=3)
    ex = LLMExecutor(config=_cfg(MAX_TOKENS=300), provider_obj=prov)
    agg = ResultAggregator(executor=ex, max_tokens_per_batch=1500)
    chunks = _chunks(9)
    groups = agg.stream_plan(chunks)
    n = len(groups)
    recs, l1 = asyncio.run(ex.process_chunks_streamed(chunks, "{transcript}", groups,
                                                      lambda g, rs: agg.level1_request(g, n, rs)))
    r = asyncio.run(agg.aggregate(recs, level1=(groups, l1)))
    assert r["plan"]["levels"] == 1 and r["plan"]["calls"] == [1] and "level1_streamed" not in r["plan"]
    assert prov.batches[-1] == ["reduce_final"] or prov.batches[-1] == ["reduce"]
