"""The OpenAI / Anthropic-compatible HTTP front-end (serve.py) on CPU: a tiny-model engine behind uvicorn
on 127.0.0.1; the package's own hosted-API providers (the reference's request shapes,
/root/reference/llm_executor.py:283-297, :376-382) pointed at it get the same completion as the
in-process engine; concurrent clients share engine batches; bad requests / keys are refused."""
import asyncio
import json
import os
import socket
import subprocess
import sys
import threading
import time
import urllib.error
import urllib.request
from concurrent.futures import ThreadPoolExecutor

import pytest

uvicorn = pytest.importorskip("uvicorn")
pytest.importorskip("fastapi")

from llm_map_reduce_summarizer_amd.config import LLMConfig  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider  # noqa: E402
from llm_map_reduce_summarizer_amd.pipeline.providers import (AnthropicProvider, GenRequest,  # noqa: E402
                                                              OpenAIProvider)
from llm_map_reduce_summarizer_amd.serve import (ContinuousBatcher, anthropic_request, build_app,  # noqa: E402
                                                 make_batcher, openai_request)

KEY = "sk-local-test"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def server():
    provider = LocalEngineProvider("tiny-gqa4", LLMConfig(), device="cpu", use_graphs=False, max_model_len=2048)
    batcher = make_batcher(provider, max_batch=16, window_s=0.2)
    assert isinstance(batcher, ContinuousBatcher)
    batcher.start()
    app = build_app(batcher, "mrsum-tiny", api_key=KEY)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 30:
        time.sleep(0.05)
    assert srv.started
    yield provider, batcher, "http://127.0.0.1:%d" % port
    srv.should_exit = True
    th.join(10)
    batcher.shutdown(10)


def _post(url, body, key=KEY, anthropic=False):
    headers = {"Content-Type": "application/json"}
    if key:
        headers.update({"x-api-key": key} if anthropic else {"Authorization": "Bearer " + key})
    req = urllib.request.Request(url, data=json.dumps(body).encode(), headers=headers, method="POST")
    try:
        with urllib.request.urlopen(req, timeout=120) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def test_openai_provider_through_server_matches_engine(server):
    provider, _, base = server
    cfg = LLMConfig(OPENAI_BASE_URL=base + "/v1", OPENAI_API_KEY=KEY)
    req = GenRequest(user="Summarize: the meeting moved to Tuesday.", system="You are terse.", max_tokens=7,
                     temperature=0.3)
    via_http = asyncio.run(OpenAIProvider("mrsum-tiny", cfg).generate(req))
    direct = asyncio.run(provider.generate_batch([GenRequest(req.user, req.system, 7, 0.3, stage="serve")]))[0]
    assert via_http.text == direct.text
    assert (via_http.prompt_tokens, via_http.completion_tokens) == (direct.prompt_tokens, 7)


def test_anthropic_provider_through_server(server):
    provider, _, base = server
    cfg = LLMConfig(ANTHROPIC_BASE_URL=base + "/v1", ANTHROPIC_API_KEY=KEY)
    req = GenRequest(user="List three colours.", system="Answer briefly.", max_tokens=5, temperature=0.0)
    res = asyncio.run(AnthropicProvider("mrsum-tiny", cfg).generate(req))
    direct = asyncio.run(provider.generate_batch([GenRequest(req.user, req.system, 5, 0.0, stage="serve")]))[0]
    assert res.text == direct.text and res.completion_tokens == 5


def test_concurrent_clients_share_batches(server):
    _, batcher, base = server
    before = dict(batcher.stats)
    bodies = [{"model": "x", "messages": [{"role": "user", "content": "request %d" % i}], "max_tokens": 4,
               "temperature": 0.5} for i in range(6)]
    with ThreadPoolExecutor(6) as ex:
        outs = list(ex.map(lambda b: _post(base + "/v1/chat/completions", b), bodies))
    assert all(st == 200 for st, _ in outs)
    for _, o in outs:
        assert o["object"] == "chat.completion" and o["choices"][0]["message"]["role"] == "assistant"
        assert o["usage"]["completion_tokens"] == 4 and o["choices"][0]["finish_reason"] == "length"
    assert batcher.stats["requests"] - before["requests"] == 6
    assert batcher.stats["batches"] - before["batches"] < 6  # the window collected several per batch


def test_late_request_joins_running_generate(server):
    """Continuous batching across HTTP requests: a short request sent while a long one decodes joins the
    running engine batch (feeder) and is answered before the long one finishes."""
    provider, batcher, base = server
    fed0 = provider.engine.stats.get("fed_requests", 0)
    calls0 = batcher.stats["batches"]
    done = {}

    def send(name, n, delay):
        time.sleep(delay)
        st, out = _post(base + "/v1/chat/completions",
                        {"messages": [{"role": "user", "content": name}], "max_tokens": n})
        assert st == 200 and out["usage"]["completion_tokens"] == n
        done[name] = time.perf_counter()
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(lambda a: send(*a), [("long request", 96, 0.0), ("short request", 3, 0.6)]))
    assert done["short request"] < done["long request"]
    assert provider.engine.stats.get("fed_requests", 0) > fed0
    assert batcher.stats["batches"] - calls0 == 1  # one engine generate served both


def test_streaming_request_joins_non_streaming_generate(server):
    """A streaming client whose request joins (feeder) a generate that started with no streaming request
    still gets deltas at the sync points, not one event at the end."""
    provider, batcher, base = server
    calls0 = batcher.stats["batches"]
    out = {}

    def long():
        out["long"] = _post(base + "/v1/chat/completions",
                            {"messages": [{"role": "user", "content": "long one"}], "max_tokens": 160})

    def streamed():
        time.sleep(0.6)
        body = {"messages": [{"role": "user", "content": "streamed late"}], "max_tokens": 48, "stream": True}
        req = urllib.request.Request(base + "/v1/chat/completions", data=json.dumps(body).encode(),
                                     headers={"Authorization": "Bearer " + KEY, "Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            out["events"] = [ln for ln in r.read().decode().splitlines() if ln.startswith("data: ")]
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(lambda f: f(), [long, streamed]))
    assert out["long"][0] == 200
    assert batcher.stats["batches"] - calls0 == 1  # the streaming request joined the running generate
    chunks = [json.loads(e[6:]) for e in out["events"][:-1]]
    deltas = [c["choices"][0]["delta"].get("content", "") for c in chunks[1:-1]]
    assert len([d for d in deltas if d]) >= 2  # 48 tokens over 16-step sync windows


def test_shutdown_answers_queued_requests():
    """Requests still queued when the engine thread stops are answered with an error, and requests
    submitted after shutdown are refused at once (no client waits forever)."""
    class _Prov:
        class par:
            world = 1
        tp = 1
    b = ContinuousBatcher(_Prov(), max_batch=4)

    async def run():
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        b.q.put((GenRequest(user="queued"), loop, fut))
        b.shutdown(1)  # never started: the queue still holds the request
        r1 = await asyncio.wait_for(fut, 5)
        r2 = await b.submit(GenRequest(user="late"))
        return r1, r2
    r1, r2 = asyncio.run(run())
    assert r1.error == r2.error == "server shutting down"


def test_enqueue_after_drain_is_refused():
    """The stop check and the put are atomic against the drain: once _drain ran (even with the stop flag
    not yet set, the window of the submit / stop race), nothing can enter the queue unanswered."""
    class _Prov:
        class par:
            world = 1
        tp = 1
    b = ContinuousBatcher(_Prov(), max_batch=4)
    b._drain()
    assert not b.stop.is_set()
    assert b._enqueue(("late", None, None)) is False and b.q.empty()

    async def run():
        return await b.submit(GenRequest(user="late")), [x async for x in b.stream(GenRequest(user="late"))]
    r, st = asyncio.run(run())
    assert r.error == "server shutting down" and st[-1][1].error == "server shutting down"


def test_multi_turn_stream_models_health_metrics(server):
    _, _, base = server
    body = {"messages": [{"role": "system", "content": "s"}, {"role": "user", "content": "hi"},
                         {"role": "assistant", "content": "hello"}, {"role": "user", "content": [
                             {"type": "text", "text": "and now?"}]}], "max_tokens": 3}
    st, out = _post(base + "/v1/chat/completions", body)
    assert st == 200 and out["usage"]["completion_tokens"] == 3
    # streaming: content deltas at the engine's sync points; their concatenation is the completion
    sbody = dict(body, max_tokens=40)
    st, full = _post(base + "/v1/chat/completions", sbody)
    req = urllib.request.Request(base + "/v1/chat/completions", data=json.dumps(dict(sbody, stream=True)).encode(),
                                 headers={"Authorization": "Bearer " + KEY, "Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=120) as r:
        events = [ln for ln in r.read().decode().splitlines() if ln.startswith("data: ")]
    assert events[-1] == "data: [DONE]"
    chunks = [json.loads(e[6:]) for e in events[:-1]]
    assert all(c["object"] == "chat.completion.chunk" for c in chunks)
    assert chunks[0]["choices"][0]["delta"]["role"] == "assistant"
    deltas = [c["choices"][0]["delta"].get("content", "") for c in chunks[1:-1]]
    assert len([d for d in deltas if d]) >= 2  # 40 tokens = 3 sync points of 16 steps
    assert "".join(deltas) == full["choices"][0]["message"]["content"]
    assert chunks[-1]["choices"][0]["finish_reason"] == "length" and chunks[-1]["usage"]["completion_tokens"] == 40
    models = json.loads(urllib.request.urlopen(base + "/v1/models", timeout=30).read())
    assert models["data"][0]["id"] == "mrsum-tiny"
    health = json.loads(urllib.request.urlopen(base + "/health", timeout=30).read())
    assert health["status"] == "ok" and health["requests"] >= 1
    metrics = urllib.request.urlopen(base + "/metrics", timeout=30).read().decode()
    assert "mrsum_requests" in metrics and "mrsum_completion_tokens" in metrics


def test_refusals(server):
    _, _, base = server
    ok = {"messages": [{"role": "user", "content": "x"}], "max_tokens": 2}
    assert _post(base + "/v1/chat/completions", ok, key="wrong")[0] == 401
    assert _post(base + "/v1/chat/completions", dict(ok, n=2))[0] == 400
    assert _post(base + "/v1/chat/completions", dict(ok, stop=["\n"]))[0] == 400
    assert _post(base + "/v1/chat/completions", {"messages": []})[0] == 400
    assert _post(base + "/v1/messages", {"messages": [{"role": "assistant", "content": "x"}], "max_tokens": 2},
                 anthropic=True)[0] == 400


def test_request_mapping():
    r = openai_request({"messages": [{"role": "developer", "content": "sys"}, {"role": "user", "content": "u"}],
                        "max_completion_tokens": 9, "temperature": 0})
    assert (r.system, r.user, r.max_tokens, r.temperature, r.messages) == ("sys", "u", 9, 0.0, None)
    a = anthropic_request({"system": [{"type": "text", "text": "S"}], "messages": [{"role": "user", "content": "U"}],
                           "max_tokens": 4})
    assert (a.system, a.user, a.messages) == ("S", "U", None)
    m = anthropic_request({"messages": [{"role": "user", "content": "a"}, {"role": "assistant", "content": "b"},
                                        {"role": "user", "content": "c"}], "max_tokens": 4})
    assert [t["role"] for t in m.messages] == ["user", "assistant", "user"]


WORLD2 = r"""
import asyncio, json, os, sys, threading, time, urllib.request
from concurrent.futures import ThreadPoolExecutor
sys.path.insert(0, %(root)r)
from llm_map_reduce_summarizer_amd.parallel import dist as pdist
pdist.init_distributed_from_env(backend="gloo")
import uvicorn
from llm_map_reduce_summarizer_amd.config import LLMConfig
from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
from llm_map_reduce_summarizer_amd.serve import Batcher, build_app, follower_loop
prov = LocalEngineProvider("tiny-gqa4", LLMConfig(), device="cpu", use_graphs=False, max_model_len=2048,
                           parallel=os.environ["PAR"])
prov.warm()
batcher = Batcher(prov, max_batch=16, window_s=0.3)
if prov.par.rank != 0:
    follower_loop(prov)
    pdist.shutdown()
    sys.exit(0)
batcher.start()
srv = uvicorn.Server(uvicorn.Config(build_app(batcher, "m"), host="127.0.0.1", port=int(os.environ["HTTP_PORT"]),
                                    log_level="warning"))
th = threading.Thread(target=srv.run, daemon=True)
th.start()
while not srv.started:
    time.sleep(0.05)
def post(i):
    body = {"messages": [{"role": "user", "content": "request %%d" %% i}], "max_tokens": 5, "temperature": 0.7}
    r = urllib.request.Request("http://127.0.0.1:%%s/v1/chat/completions" %% os.environ["HTTP_PORT"],
                               data=json.dumps(body).encode(), headers={"Content-Type": "application/json"})
    return json.loads(urllib.request.urlopen(r, timeout=300).read())["choices"][0]["message"]["content"]
with ThreadPoolExecutor(4) as ex:
    texts = list(ex.map(post, range(4)))
srv.should_exit = True
th.join(30)
batcher.shutdown(60)
print("RESULT " + json.dumps({"texts": texts, "stats": batcher.stats, "plan": prov.stage_plan}), flush=True)
pdist.shutdown()
"""


@pytest.mark.parametrize("par", ["dp", "tp"])
def test_world2_server_broadcasts_batches(par):
    """torchrun-style world 2 over gloo: rank 0 serves HTTP and broadcasts each batch (and idle heartbeats),
    rank 1 runs the same SPMD generate_batch (DP replicas or one TP=2 engine); the completions equal the
    single-process engine's (per-request seeds; the CPU reference path is batch-invariant)."""
    def free():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free()), WORLD_SIZE="2", OMP_NUM_THREADS="2",
               HTTP_PORT=str(free()), PAR=par)
    procs = [subprocess.Popen([sys.executable, "-c", WORLD2 % {"root": ROOT}], env=dict(env, RANK=str(r),
                              LOCAL_RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(2)]
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (_, err) in zip(procs, outs):
        assert p.returncode == 0, err[-3000:]
    res = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("RESULT ")][-1][7:])
    assert res["stats"]["requests"] == 4 and res["stats"]["errors"] == 0
    assert res["plan"]["serve"]["tp"] == (2 if par == "tp" else 1)
    prov = LocalEngineProvider("tiny-gqa4", LLMConfig(), device="cpu", use_graphs=False, max_model_len=2048)
    direct = asyncio.run(prov.generate_batch([GenRequest("request %d" % i, None, 5, 0.7, stage="serve")
                                              for i in range(4)]))
    if par == "dp":
        assert res["texts"] == [d.text for d in direct]
    else:  # TP=2 sums the sharded products in another order: same token counts, text may differ
        assert all(isinstance(t, str) for t in res["texts"])


@pytest.mark.gpu
def test_server_on_gpu_engine():
    """The same front-end over the HIP engine on cuda:0 (decode hipGraphs on): an OpenAI-shaped request
    through HTTP returns the in-process engine's completion."""
    import torch
    assert torch.cuda.is_available()
    provider = LocalEngineProvider("tiny-gqa4", LLMConfig(), device="cuda:0", max_model_len=2048)
    batcher = make_batcher(provider, max_batch=8, window_s=0.05)
    batcher.start()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(build_app(batcher, "m"), host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    try:
        t0 = time.time()
        while not srv.started and time.time() - t0 < 30:
            time.sleep(0.05)
        cfg = LLMConfig(OPENAI_BASE_URL="http://127.0.0.1:%d/v1" % port, OPENAI_API_KEY="x")
        req = GenRequest(user="Summarize the call.", system="Be brief.", max_tokens=8, temperature=0.3)
        via_http = asyncio.run(OpenAIProvider("m", cfg).generate(req))
        direct = asyncio.run(provider.generate_batch([GenRequest(req.user, req.system, 8, 0.3, stage="serve")]))[0]
        assert via_http.text == direct.text and via_http.completion_tokens == 8
    finally:
        srv.should_exit = True
        th.join(10)
        batcher.shutdown(10)
