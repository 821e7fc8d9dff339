"""Multi-rank paths of an 8-GPU node, rehearsed on CPU ranks over gloo.

* DP at world 4 / 8 on the ``tiny-kv8`` preset (8 KV heads): summaries bit-equal to world 1, the
  LPT owner maps identical on every rank and balanced;
* TP = 4 / 8 engines (one or two KV heads per rank, 16032-row vocab shards): every rank samples the
  same tokens, and they agree with TP = 1 up to a bf16 near-tie;
* all stages on one TP = 8 engine with the 8-way KV hand-off all-to-all, and reduce-only TP = 4: the
  stage plans are asserted;
* collective-safe failures: an engine fault injected on ONE rank (one-shot, and persistent) -- every
  rank ends with identical results (summaries or identical ``[Error processing chunk: ...]`` records),
  no index-space mix-up, and no collective hang (the run ends within the retry budget).
Reference fan-out / barrier: ``llm_executor.py:133-157``, ``result_aggregator.py:321-342``.
"""

import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PIPE = textwrap.dedent("""
    import asyncio, json, os, sys, time
    sys.path.insert(0, %(root)r)
    from llm_map_reduce_summarizer_amd.parallel import dist as pdist
    pdist.init_distributed_from_env(backend="gloo", timeout_s=120)
    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.pipeline.executor import LLMExecutor
    from llm_map_reduce_summarizer_amd.pipeline.orchestrator import TranscriptSummarizer
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    opt = json.loads(os.environ["OPT"])
    if opt.get("force_handoff"):
        # the tiny preset's KV (128-dim heads) outweighs its 512-wide activations, so the cost model keeps
        # its single-prompt stage on the TP forward; Llama-3 goes context-parallel (tests/test_plan.py)
        LocalEngineProvider._handoff_pays = lambda self, prompts, reqs, k=None: self.handoff and bool(reqs)
    if opt.get("oom_export_rank") == int(os.environ.get("RANK", 0)):
        # this rank's DP engine cannot hold its share of a hand-off prefill (KV pool exhausted)
        from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine
        def _oom(self, *a, **k):
            raise MemoryError("cannot admit any request: KV cache too small (injected)")
        LLMEngine.prefill_export = _oom
    cfg = LLMConfig(MAX_TOKENS=6, RETRY_DELAY=0.05)
    prov = LocalEngineProvider(opt.get("model", "tiny-kv8"), cfg, device="cpu", max_model_len=4096,
                               engine_options={"kv_pages": 512, "max_num_seqs": 16},
                               parallel=opt.get("parallel", "dp"), fault_inject=opt.get("fault"))
    ex = LLMExecutor(config=cfg, provider_obj=prov)
    summ = TranscriptSummarizer(executor=ex, max_tokens_per_chunk=1000,
                                aggregator_options={"max_tokens_per_batch": 40})
    cap = {}
    orig = ex.process_chunks
    async def capture(*a, **k):
        r = await orig(*a, **k)
        cap["s"] = [c["summary"] for c in r]
        return r
    ex.process_chunks = capture
    t0 = time.time()
    rep = asyncio.run(summ.summarize(synthetic_transcript(opt.get("hours", 0.5), seed=3)))
    st = prov.stats()
    tpe = st.get("tp_engines", {})
    out = {"rank": int(os.environ.get("RANK", 0)), "summary": rep["summary"], "chunks": rep["chunks"],
           "imported_groups": sum(e.get("imported_prefills", 0) for e in tpe.values()),
           "cp_all": st.get("cp_prefills", 0),
           "plan": {k: rep["reduce_plan"][k] for k in ("levels", "calls")},
           "chunk_summaries": cap["s"],
           "failed": ex.failed_requests, "retried": ex.retried_requests, "owner_maps": prov.owner_maps, "stage_plan": st.get("stage_plan", {}),
           "imported": st.get("tp_engine", {}).get("imported_prefills", 0), "cp": st.get("cp_prefills", 0),
           "handoff_fallbacks": st.get("handoff_fallbacks", 0),
           "seconds": time.time() - t0}
    print("RESULT " + json.dumps(out), flush=True)
    pdist.shutdown()
""")


def _launch(code, world, env_extra, timeout=900):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               OMP_NUM_THREADS="1", **env_extra)
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            o, err = p.communicate(timeout=timeout)
            assert p.returncode == 0, err[-3000:]
            outs.append(json.loads([line for line in o.splitlines() if line.startswith("RESULT ")][-1][7:]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


def _pipe(world, **opt):
    return _launch(PIPE % {"root": ROOT}, world, {"OPT": json.dumps(opt)})


@pytest.fixture(scope="module")
def single():
    return _pipe(1)[0]


def _check_owner_maps(outs):
    from llm_map_reduce_summarizer_amd.engine.provider import assign_balanced  # noqa: F401
    maps = [o["owner_maps"] for o in outs]
    assert all(m == maps[0] for m in maps), "ranks disagree on the request -> replica assignment"
    world = len(outs)
    for stage, calls in maps[0].items():
        for owner in calls:
            assert set(owner) <= set(range(world))
            if len(owner) >= world:
                assert len(set(owner)) == world, (stage, owner)  # every replica gets work


@pytest.mark.parametrize("world", [4, 8])
def test_dp_world_equals_single(single, world):
    outs = _pipe(world)
    assert single["chunks"] >= 8 and single["plan"]["levels"] >= 2
    for o in outs:
        assert o["summary"] == single["summary"]
        assert o["chunk_summaries"] == single["chunk_summaries"]
        assert o["plan"] == single["plan"]
    _check_owner_maps(outs)


def test_all_stages_tp8_with_handoff():
    outs = _pipe(8, parallel="tp", force_handoff=True)
    assert all(o["summary"] == outs[0]["summary"] for o in outs)
    assert outs[0]["imported"] > 0  # TP stages prefilled data-parallel, KV moved by the 8-way all-to-all
    for stage, plan in outs[0]["stage_plan"].items():
        assert plan["tp"] == 8, (stage, plan)
    assert outs[0]["stage_plan"]["map"]["handoff"] is True
    # the single-prompt final reduce prefilled context-parallel over the 8 ranks (no one-rank prefill)
    assert outs[0]["stage_plan"]["reduce_final"]["handoff"] is True and all(o["cp"] >= 1 for o in outs)


def test_per_stage_layouts_tp2_tp4_tp8(single):
    """One world-8 job with a different TP x DP layout per stage: map on 4 replicas of a TP=2 engine,
    level-1 reduce on 2 replicas of a TP=4 engine, the final reduce on one TP=8 engine (each group
    prefilling its share data-parallel / context-parallel and importing the KV).  Every rank ends with
    the same summary; the chunk summaries match world 1 up to bf16 near-ties of the sharded sums."""
    outs = _pipe(8, parallel="map:tp2,reduce_l1:tp4,reduce_final:tp8", force_handoff=True)
    assert all(o["summary"] == outs[0]["summary"] for o in outs)
    assert all(o["chunk_summaries"] == outs[0]["chunk_summaries"] for o in outs)
    sp = outs[0]["stage_plan"]
    assert sp["map"]["tp"] == 2 and sp["reduce_l1"]["tp"] == 4 and sp["reduce_final"]["tp"] == 8, sp
    assert outs[0]["plan"] == single["plan"]
    same = sum(a == b for a, b in zip(outs[0]["chunk_summaries"], single["chunk_summaries"]))
    assert same >= len(single["chunk_summaries"]) // 2, (same, len(single["chunk_summaries"]))
    assert outs[0]["imported_groups"] > 0 or outs[0]["imported"] > 0
    maps = [o["owner_maps"] for o in outs]
    assert all(m == maps[0] for m in maps), "ranks disagree on the request -> TP group assignment"
    for owner in maps[0]["map"]:  # 4 TP=2 groups, each with work
        assert set(owner) == {0, 1, 2, 3}, owner


def test_reduce_tp4_map_dp4():
    outs = _pipe(4, parallel="reduce_tp")
    assert all(o["summary"] == outs[0]["summary"] for o in outs)
    sp = outs[0]["stage_plan"]
    assert sp["map"]["tp"] == 1 and sp["reduce_final"]["tp"] == 4, sp
    _check_owner_maps(outs)


TP_ENGINE = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, %(root)r)
    from llm_map_reduce_summarizer_amd.parallel import dist as pdist
    pdist.init_distributed_from_env(backend="gloo", timeout_s=120)
    par = pdist.setup_parallel(int(os.environ.get("TP", "1")))
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    eng = LLMEngine(get_model_config("tiny-kv8", init_std=0.05), device="cpu", max_model_len=512, max_num_seqs=4,
                    kv_pages=64, sync_every=3, tp_rank=par.tp_rank, tp_size=par.tp, tp_group=par.tp_group)
    assert eng.model.hkv == 8 // par.tp and eng.model.vocab_local == 128256 // par.tp
    prompts = [[128000] + [(i * 7 + j * 3) %% 9000 + 5 for j in range(20 + 9 * i)] for i in range(3)]
    outs = eng.generate(prompts, [SamplingParams(5, 0.0, i) for i in range(3)])
    print("RESULT " + json.dumps([o.token_ids for o in outs]), flush=True)
    pdist.shutdown()
""")


@pytest.mark.parametrize("tp", [4, 8])
def test_tp_engine_matches_tp1(tp):
    code = TP_ENGINE % {"root": ROOT}
    ref = _launch(code, 1, {"TP": "1"})[0]
    outs = _launch(code, tp, {"TP": str(tp)})
    assert all(o == outs[0] for o in outs)  # every TP rank samples the same tokens
    same = sum(a == b for a, b in zip(outs[0], ref))
    assert same >= 2, (outs[0], ref)  # greedy; a bf16 near-tie may flip one sequence


@pytest.mark.parametrize("world", [2, 4])
def test_one_shot_fault_on_one_rank_recovers(single, world):
    t0 = time.time()
    outs = _pipe(world, fault="1:1")
    assert time.time() - t0 < 600
    for o in outs:
        assert o["summary"] == single["summary"], "a retried request must produce the same summary"
        assert o["chunk_summaries"] == single["chunk_summaries"]
        assert o["failed"] == 0 and o["retried"] > 0
    _check_owner_maps(outs)


@pytest.mark.parametrize("world", [2, 4])
def test_persistent_fault_on_one_rank_is_consistent(world):
    outs = _pipe(world, fault="1:-1")
    ref = outs[0]
    for o in outs:
        assert o["chunk_summaries"] == ref["chunk_summaries"]
        assert o["summary"] == ref["summary"]
        assert o["failed"] == ref["failed"]
        assert o["seconds"] < 300, "a rank waited on a collective its peer never entered"
    errs = [s for s in ref["chunk_summaries"] if s.startswith("[Error processing chunk:")]
    # retries re-balance the failed requests over the replicas: some land on healthy ranks and succeed,
    # the ones that keep landing on the sick rank end as error records -- identically on every rank
    assert ref["retried"] > 0 and len(errs) < len(ref["chunk_summaries"])
    assert all(o["retried"] == ref["retried"] for o in outs)
    assert all("injected engine fault on rank 1" in s for s in errs)
    _check_owner_maps(outs)


CP_ENGINE = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, %(root)r)
    import torch
    from llm_map_reduce_summarizer_amd.parallel import dist as pdist
    pdist.init_distributed_from_env(backend="gloo", timeout_s=120)
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import ImportedPrefill, LLMEngine, SamplingParams
    cfg = get_model_config("tiny-kv8", init_std=0.05)
    full = LLMEngine(cfg, device="cpu", max_model_len=1024, max_num_seqs=4, kv_pages=64, sync_every=3)
    tp = LLMEngine(cfg, device="cpu", max_model_len=1024, max_num_seqs=4, kv_pages=64, sync_every=3,
                   tp_rank=rank, tp_size=world, tp_group=pdist.tp_group_for(world))
    prompt = [128000] + [(j * 37) %% 9000 + 5 for j in range(301)]
    sp = SamplingParams(6, 0.0, 0)
    first, kv = full.prefill_export_cp(prompt, sp, rank, world, group=pdist.tp_group_for(world))
    # reference: the one-rank prefill_export of the same prompt (this rank's KV heads)
    f1, packs = full.prefill_export([prompt], [sp], world)
    ref = packs[rank].view(kv.shape)
    err = float((kv.float() - ref.float()).abs().max())
    cp_out = tp.generate([prompt], [sp], imported={0: ImportedPrefill(first, kv)})[0].token_ids
    one = full.generate([prompt], [sp])[0].token_ids
    print("RESULT " + json.dumps({"first": first, "f1": f1[0], "kv_err": err, "cp": cp_out, "one": one,
                                  "free": full.kv.alloc.available(), "pages": full.kv.num_pages,
                                  "cp_prefills": full.stats.get("cp_prefills", 0)}), flush=True)
    pdist.shutdown()
""")


@pytest.mark.parametrize("world", [2, 4])
def test_context_parallel_prefill_matches_one_rank_prefill(world):
    """Context-parallel prefill (zigzag slices per rank, per-layer K/V all-gather): every rank ends with
    the same KV heads a one-rank prefill exports to it, the same first token, and the TP decode from it
    generates what the TP=1 engine does (greedy; bf16 rounding of the slice order may flip a near-tie)."""
    outs = _launch(CP_ENGINE % {"root": ROOT}, world, {})
    for o in outs:
        assert o["cp_prefills"] == 1 and o["free"] == o["pages"] - 1  # pages returned
        assert o["kv_err"] < 0.05, o["kv_err"]
        assert o["first"] == o["f1"] == outs[0]["first"]
        assert o["cp"] == outs[0]["cp"]  # every TP rank samples the same tokens
    same = sum(a == b for a, b in zip(outs[0]["cp"], outs[0]["one"]))
    assert same >= len(outs[0]["one"]) - 1 or outs[0]["cp"][:3] == outs[0]["one"][:3], outs[0]


def test_handoff_kv_exhaustion_falls_back_to_tp_prefill():
    """A hand-off prefill that does not fit one rank's DP KV pool (MemoryError on rank 1 only): the TP=2 group of
    that rank agrees and lets its TP engine prefill the prompts itself -- no failed request, the other group
    keeps its hand-off, every rank ends with the same summary (round-6 rehearsal finding: 1 % KV pools)."""
    outs = _pipe(4, parallel="map:tp2,reduce_final:tp4", oom_export_rank=1)
    assert all(o["failed"] == 0 for o in outs), [o["failed"] for o in outs]
    assert len({o["summary"] for o in outs}) == 1 and outs[0]["summary"]
    fb = [o["handoff_fallbacks"] for o in outs]
    assert fb[0] > 0 and fb[1] > 0 and fb[0] == fb[1], fb  # ranks 0, 1: the group with the exhausted pool
    assert fb[2] == fb[3] == 0, fb
