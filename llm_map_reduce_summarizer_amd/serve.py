"""OpenAI- and Anthropic-compatible HTTP front-end for the on-node engine.

The reference's only process boundary is an HTTPS POST to a hosted model (``/root/reference/
llm_executor.py:283-297`` ``/v1/chat/completions``, ``:376-382`` ``/v1/messages``).  This server puts the
MI355X engine behind those two endpoints, so anything that speaks them -- the reference itself with
``OPENAI_BASE_URL`` pointed here, this package's ``--provider openai|anthropic``, any OpenAI client --
runs on the local GPUs unchanged:

    python -m llm_map_reduce_summarizer_amd.serve --model llama3-8b --port 8000
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m llm_map_reduce_summarizer_amd.serve ...

Endpoints: ``POST /v1/chat/completions``, ``POST /v1/messages``, ``GET /v1/models``, ``GET /health``,
``GET /metrics`` (Prometheus text).  ``stream: true`` on the chat endpoint streams
``chat.completion.chunk`` events as the engine produces tokens (every host sync point, 16 decode steps)
on a single-process engine, the whole completion as one event under torchrun; Anthropic streaming gets the
message as one event.  Stop sequences and n > 1 are not supported (400).

Batching: HTTP handlers only enqueue; one engine thread owns the engine.  Single process
(``ContinuousBatcher``): the first requests start a generate and every request that arrives while it runs
joins the running batch at the next host sync point (the engine's feeder hook) -- continuous batching
with paged KV and the decode hipGraphs; each client is answered when its own sequence finishes.  Under
torchrun (``Batcher``): rank 0 collects for ``--batch-window-ms`` (up to ``--max-batch``) and broadcasts
every batch (or an idle heartbeat, so peers never sit in a collective past its timeout) to the other
ranks, which all run the same SPMD ``generate_batch`` -- DP replicas or TP engines chosen by the
summarizer's stage planner.
"""

import argparse
import asyncio
import hmac
import json
import logging
import os
import queue
import threading
import time
import uuid
from dataclasses import asdict
from typing import Any, Dict, List, Optional, Tuple

from .config import LLMConfig
from .parallel import dist as pdist
from .pipeline.providers import GenRequest, GenResult

log = logging.getLogger("mrsum.serve")

HEARTBEAT_S = 1.0  # multi-rank: idle broadcast period


class BadRequest(ValueError):
    pass


def _text(content: Any) -> str:
    """OpenAI / Anthropic message content: a string or a list of parts ({"type": "text", "text": ...})."""
    if isinstance(content, str):
        return content
    if isinstance(content, list):
        out = []
        for part in content:
            if isinstance(part, dict) and part.get("type") == "text":
                out.append(str(part.get("text", "")))
            elif isinstance(part, str):
                out.append(part)
            else:
                raise BadRequest("only text content parts are supported")
        return "".join(out)
    raise BadRequest("message content must be a string or a list of text parts")


def _common(body: Dict[str, Any], default_temp: float) -> Tuple[int, float]:
    if body.get("stop"):
        raise BadRequest("stop sequences are not supported")
    if int(body.get("n", 1) or 1) != 1:
        raise BadRequest("n > 1 is not supported")
    mt = body.get("max_completion_tokens", body.get("max_tokens"))
    max_tokens = int(mt) if mt is not None else 1000
    if max_tokens < 1:
        raise BadRequest("max_tokens must be >= 1")
    temp = body.get("temperature")
    return max_tokens, float(default_temp if temp is None else temp)


def openai_request(body: Dict[str, Any], default_temp: float = 1.0) -> GenRequest:
    """GenRequest of an OpenAI ``/v1/chat/completions`` body.  A [system?, user] chat keeps the
    reference's request shape (same prompt rendering and seed as the in-process provider)."""
    msgs = body.get("messages")
    if not isinstance(msgs, list) or not msgs:
        raise BadRequest("messages must be a non-empty list")
    turns = []
    for m in msgs:
        role = m.get("role") if isinstance(m, dict) else None
        if role == "developer":
            role = "system"
        if role not in ("system", "user", "assistant"):
            raise BadRequest("unsupported message role %r" % role)
        turns.append({"role": role, "content": _text(m.get("content", ""))})
    max_tokens, temp = _common(body, default_temp)
    roles = [t["role"] for t in turns]
    if roles in (["user"], ["system", "user"]):
        return GenRequest(user=turns[-1]["content"], system=turns[0]["content"] if len(turns) == 2 else None,
                          max_tokens=max_tokens, temperature=temp, stage="serve")
    return GenRequest(user=turns[-1]["content"], max_tokens=max_tokens, temperature=temp, stage="serve",
                      messages=turns)


def anthropic_request(body: Dict[str, Any], default_temp: float = 1.0) -> GenRequest:
    """GenRequest of an Anthropic ``/v1/messages`` body (top-level ``system``)."""
    msgs = body.get("messages")
    if not isinstance(msgs, list) or not msgs:
        raise BadRequest("messages must be a non-empty list")
    system = body.get("system")
    system = _text(system) if system else None
    turns = [{"role": "system", "content": system}] if system else []
    for m in msgs:
        role = m.get("role") if isinstance(m, dict) else None
        if role not in ("user", "assistant"):
            raise BadRequest("unsupported message role %r" % role)
        turns.append({"role": role, "content": _text(m.get("content", ""))})
    max_tokens, temp = _common(body, default_temp)
    if [t["role"] for t in turns[-1:]] != ["user"]:
        raise BadRequest("the last message must be from the user")
    if len(msgs) == 1:
        return GenRequest(user=turns[-1]["content"], system=system, max_tokens=max_tokens, temperature=temp,
                          stage="serve")
    return GenRequest(user=turns[-1]["content"], max_tokens=max_tokens, temperature=temp, stage="serve",
                      messages=turns)


def _finish(res: GenResult) -> str:
    return "length" if (res.extra or {}).get("finish_reason") == "length" else "stop"


def openai_response(res: GenResult, model: str) -> Dict[str, Any]:
    return {"id": "chatcmpl-" + uuid.uuid4().hex[:24], "object": "chat.completion", "created": int(time.time()),
            "model": model,
            "choices": [{"index": 0, "message": {"role": "assistant", "content": res.text},
                         "finish_reason": _finish(res)}],
            "usage": {"prompt_tokens": res.prompt_tokens, "completion_tokens": res.completion_tokens,
                      "total_tokens": res.prompt_tokens + res.completion_tokens}}


def anthropic_response(res: GenResult, model: str) -> Dict[str, Any]:
    return {"id": "msg_" + uuid.uuid4().hex[:24], "type": "message", "role": "assistant", "model": model,
            "content": [{"type": "text", "text": res.text}],
            "stop_reason": "max_tokens" if _finish(res) == "length" else "end_turn", "stop_sequence": None,
            "usage": {"input_tokens": res.prompt_tokens, "output_tokens": res.completion_tokens}}


class Batcher:
    """Request queue -> batches -> ``provider.generate_batch`` on one engine thread (see module doc)."""

    def __init__(self, provider, max_batch: int = 64, window_s: float = 0.005):
        self.provider = provider
        self.max_batch = max(1, int(max_batch))
        self.window_s = max(0.0, float(window_s))
        self.q: "queue.Queue[Tuple[GenRequest, asyncio.AbstractEventLoop, asyncio.Future]]" = queue.Queue()
        self.stop = threading.Event()
        self.stats = {"requests": 0, "batches": 0, "errors": 0, "prompt_tokens": 0, "completion_tokens": 0,
                      "engine_s": 0.0, "max_batch_seen": 0}
        self._thread: Optional[threading.Thread] = None
        # enqueue vs drain: once _drain has closed the queue no request may enter it (its client would wait
        # on its future forever), so the closed check and the put happen under the lock _drain takes
        self._qlock = threading.Lock()
        self._closed = False

    def _enqueue(self, item) -> bool:
        """Queue ``item`` unless the server is stopping / drained (False: answer the client yourself)."""
        with self._qlock:
            if self._closed or self.stop.is_set():
                return False
            self.q.put(item)
            return True

    async def submit(self, req: GenRequest) -> GenResult:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        if not self._enqueue((req, loop, fut)):
            return GenResult("", error="server shutting down")
        return await fut

    def _drain(self) -> None:
        """Answer every request still queued when the engine thread stops (its client would otherwise
        wait on its future until the process dies); no request can be queued after this."""
        with self._qlock:
            self._closed = True
        while True:
            try:
                it = self.q.get_nowait()
            except queue.Empty:
                return
            lp, fut = it[1], it[2]
            lp.call_soon_threadsafe(lambda f=fut: f.done() or f.set_result(GenResult("", error="server shutting down")))

    async def stream(self, req: GenRequest):
        """Async iterator of ("delta", text) items, then ("done", GenResult).  Windowed batches (multi-rank)
        deliver the whole completion as one delta; the continuous batcher streams at every sync point."""
        res = await self.submit(req)
        if not res.error and res.text:
            yield "delta", res.text
        yield "done", res

    def _collect(self, first_timeout: float):
        try:
            items = [self.q.get(timeout=first_timeout)]
        except queue.Empty:
            return []
        deadline = time.perf_counter() + self.window_s
        while len(items) < self.max_batch:
            left = deadline - time.perf_counter()
            try:
                items.append(self.q.get(timeout=max(0.0, left)) if left > 0 else self.q.get_nowait())
            except queue.Empty:
                break
        return items

    def run_batch(self, reqs: List[GenRequest]) -> List[GenResult]:
        t0 = time.perf_counter()
        try:
            res = asyncio.run(self.provider.generate_batch(reqs))
        except Exception as e:  # noqa: BLE001 -- every waiting client gets the error, the server lives on
            log.exception("batch of %d failed", len(reqs))
            res = [GenResult("", error="%s: %s" % (type(e).__name__, e)) for _ in reqs]
        self.stats["engine_s"] += time.perf_counter() - t0
        return res

    def loop(self) -> None:
        """Rank 0's engine thread."""
        multi = pdist.is_initialized() and self.provider.par.world > 1
        while True:
            items = [] if self.stop.is_set() else self._collect(HEARTBEAT_S if multi else 0.1)
            if multi:  # every rank enters the same collectives, heartbeat or batch
                pdist.broadcast_json({"stop": self.stop.is_set(), "reqs": [asdict(it[0]) for it in items]})
            if self.stop.is_set() and not items:
                self._drain()
                break
            if not items:
                continue
            reqs = [it[0] for it in items]
            res = self.run_batch(reqs)
            self.stats["batches"] += 1
            self.stats["requests"] += len(reqs)
            self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], len(reqs))
            for (_, lp, fut), r in zip(items, res):
                self.stats["errors"] += bool(r.error)
                self.stats["prompt_tokens"] += r.prompt_tokens
                self.stats["completion_tokens"] += r.completion_tokens
                lp.call_soon_threadsafe(lambda f=fut, v=r: f.done() or f.set_result(v))

    def start(self) -> None:
        self._thread = threading.Thread(target=self.loop, name="mrsum-engine", daemon=True)
        self._thread.start()

    def shutdown(self, timeout: Optional[float] = None) -> None:
        self.stop.set()
        if self._thread is not None:
            self._thread.join(timeout)
        self._drain()


class ContinuousBatcher(Batcher):
    """Single-process engine: requests that arrive while a generate runs JOIN it at the next host sync
    point (the engine's feeder hook, every ``sync_every`` decode steps) instead of waiting for the whole
    batch -- continuous batching across HTTP requests; each client is answered the moment its own
    sequence finishes."""

    async def stream(self, req: GenRequest):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        sq: "asyncio.Queue[str]" = asyncio.Queue()
        if not self._enqueue((req, loop, fut, sq)):
            yield "done", GenResult("", error="server shutting down")
            return
        while True:
            getter = asyncio.ensure_future(sq.get())
            await asyncio.wait([getter, fut], return_when=asyncio.FIRST_COMPLETED)
            if getter.done():
                yield "delta", getter.result()
                continue
            getter.cancel()
            while not sq.empty():
                yield "delta", sq.get_nowait()
            yield "done", fut.result()
            return

    def loop(self) -> None:
        from .engine.engine import SamplingParams
        from .engine.provider import _req_seed
        prov = self.provider
        while not self.stop.is_set():
            items = self._collect(0.1)
            if not items:
                continue
            pending: Dict[int, Any] = {}
            sent: Dict[int, int] = {}  # streamed requests: characters already sent
            nxt = [0]

            def admit(its):
                out = []
                for it in its:
                    req, lp, fut = it[:3]
                    try:
                        if req.max_tokens >= prov.max_model_len:
                            raise BadRequest("max_tokens must be below max_model_len (%d)" % prov.max_model_len)
                        ids = prov.encode_request(req)
                    except Exception as e:  # noqa: BLE001 -- this client only
                        self._resolve(lp, fut, GenResult("", error="%s: %s" % (type(e).__name__, e)))
                        continue
                    pending[nxt[0]] = it
                    if len(it) > 3:
                        sent[nxt[0]] = 0
                    nxt[0] += 1
                    out.append((ids, SamplingParams(req.max_tokens, req.temperature, _req_seed(prov.seed, req))))
                    self.stats["requests"] += 1
                return out

            def push(rid, text, final):
                """Send the new characters of a streamed request (held back: a trailing incomplete
                UTF-8 sequence, decoded as U+FFFD, until its bytes are complete)."""
                it = pending[rid]
                safe = text if final else text.rstrip("\ufffd")
                if len(safe) > sent[rid]:
                    delta, sent[rid] = safe[sent[rid]:], len(safe)
                    it[1].call_soon_threadsafe(it[3].put_nowait, delta)

            def on_sync(tok_map):
                for rid, ids in tok_map.items():
                    if rid in sent and rid in pending:
                        push(rid, prov.tokenizer.decode(ids), False)

            # asked at every sync point: a streaming request that joins later through the feeder still
            # gets its deltas, and batches with no streaming request skip the token-buffer copy
            on_sync.wanted = lambda: bool(sent)

            def finish(done):
                for rid, o in done:
                    text = prov.tokenizer.decode(o.token_ids)
                    if rid in sent:
                        push(rid, text, True)
                        sent.pop(rid)
                    req, lp, fut = pending.pop(rid)[:3]
                    self._resolve(lp, fut, GenResult(text, o.prompt_len, len(o.token_ids),
                                                     extra={"finish_reason": o.finish_reason}))

            def feeder(done):
                finish(done)
                room = self.max_batch - len(pending)
                more = []
                while room > 0 and not self.stop.is_set():
                    try:
                        more.append(self.q.get_nowait())
                    except queue.Empty:
                        break
                    room -= 1
                return admit(more)

            first = admit(items)
            if not first:
                continue
            t0 = time.perf_counter()
            self.stats["batches"] += 1
            try:
                outs = prov.engine.generate([ids for ids, _ in first], [sp for _, sp in first],
                                            ignore_eos=prov.ignore_eos, feeder=feeder, on_sync=on_sync)
                finish([(rid, o) for rid, o in enumerate(outs) if rid in pending and o is not None])
            except Exception as e:  # noqa: BLE001 -- every in-flight client gets the error
                log.exception("engine generate failed")
                for rid in list(pending):
                    req, lp, fut = pending.pop(rid)[:3]
                    self._resolve(lp, fut, GenResult("", error="%s: %s" % (type(e).__name__, e)))
            self.stats["engine_s"] += time.perf_counter() - t0
            self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], nxt[0])
        self._drain()

    def _resolve(self, lp, fut, r: GenResult) -> None:
        self.stats["errors"] += bool(r.error)
        self.stats["prompt_tokens"] += r.prompt_tokens
        self.stats["completion_tokens"] += r.completion_tokens
        lp.call_soon_threadsafe(lambda f=fut, v=r: f.done() or f.set_result(v))


def make_batcher(provider, max_batch: int = 64, window_s: float = 0.005) -> Batcher:
    """Continuous (feeder) batching for a single-process engine, windowed batches broadcast to the ranks
    otherwise (their SPMD generate needs every rank to see the same request set)."""
    if provider.par.world == 1 and provider.tp == 1:
        return ContinuousBatcher(provider, max_batch, window_s)
    return Batcher(provider, max_batch, window_s)


def follower_loop(provider) -> None:
    """Ranks > 0: run every batch rank 0 broadcasts until it says stop."""
    while True:
        msg = pdist.broadcast_json(None)
        reqs = [GenRequest(**r) for r in msg["reqs"]]
        if reqs:
            try:
                asyncio.run(provider.generate_batch(reqs))
            except Exception:  # noqa: BLE001 -- rank 0 reports; the collectives inside already matched
                log.exception("follower batch failed")
        if msg["stop"]:
            return


async def _openai_events(items, model: str):
    """Server-sent ``chat.completion.chunk`` events: the role, content deltas as the engine produces them
    (every host sync point), then finish_reason + usage, then ``[DONE]``."""
    cid, created = "chatcmpl-" + uuid.uuid4().hex[:24], int(time.time())

    def chunk(delta, finish=None, usage=None):
        c = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
             "choices": [{"index": 0, "delta": delta, "finish_reason": finish}]}
        if usage is not None:
            c["usage"] = usage
        return "data: %s\n\n" % json.dumps(c)
    yield chunk({"role": "assistant", "content": ""})
    async for kind, v in items:
        if kind == "delta":
            yield chunk({"content": v})
            continue
        if v.error:
            yield "data: %s\n\n" % json.dumps({"error": {"message": v.error, "type": "engine_error"}})
        else:
            yield chunk({}, _finish(v), {"prompt_tokens": v.prompt_tokens, "completion_tokens": v.completion_tokens,
                                         "total_tokens": v.prompt_tokens + v.completion_tokens})
    yield "data: [DONE]\n\n"


def build_app(batcher: Batcher, model_name: str, api_key: Optional[str] = None, default_temp: float = 1.0):
    """The FastAPI app (handlers enqueue on ``batcher``; ``api_key``: required Bearer / x-api-key)."""
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

    app = FastAPI(title="mrsum engine", version="1")
    started = time.time()

    def _err(status: int, msg: str, kind: str) -> JSONResponse:
        return JSONResponse({"error": {"message": msg, "type": kind}}, status_code=status)

    def _authorised(request: Request) -> bool:
        if not api_key:
            return True
        auth = request.headers.get("authorization", "")
        token = auth[7:] if auth.startswith("Bearer ") else request.headers.get("x-api-key", "")
        return hmac.compare_digest(token.encode(), api_key.encode())  # constant-time

    async def _serve(request: Request, parse, render):
        if not _authorised(request):
            return _err(401, "invalid API key", "authentication_error")
        try:
            body = await request.json()
            req = parse(body, default_temp)
        except BadRequest as e:
            return _err(400, str(e), "invalid_request_error")
        except (ValueError, TypeError, AttributeError) as e:
            return _err(400, "malformed request: %s" % e, "invalid_request_error")
        model = body.get("model") or model_name
        if body.get("stream") and render is openai_response:
            return StreamingResponse(_openai_events(batcher.stream(req), model), media_type="text/event-stream")
        res = await batcher.submit(req)
        if res.error:
            return _err(500, res.error, "engine_error")
        out = render(res, model)
        if body.get("stream"):  # Anthropic: the whole message as one event
            async def events():
                yield "data: %s\n\n" % json.dumps(out)
                yield "data: [DONE]\n\n"
            return StreamingResponse(events(), media_type="text/event-stream")
        return JSONResponse(out)

    @app.post("/v1/chat/completions")
    async def chat_completions(request: Request):
        return await _serve(request, openai_request, openai_response)

    @app.post("/v1/messages")
    async def messages(request: Request):
        return await _serve(request, anthropic_request, anthropic_response)

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "created": int(started),
                                            "owned_by": "mrsum"}]}

    @app.get("/health")
    async def health():
        return {"status": "ok", "uptime_s": round(time.time() - started, 1), **batcher.stats}

    @app.get("/metrics")
    async def metrics():
        lines = []
        for k, v in batcher.stats.items():
            kind = "gauge" if k == "max_batch_seen" else "counter"
            lines += ["# TYPE mrsum_%s %s" % (k, kind), "mrsum_%s %s" % (k, v)]
        return PlainTextResponse("\n".join(lines) + "\n", media_type="text/plain; version=0.0.4")

    return app


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", default="llama3-8b", help="engine preset (or hf with --weights)")
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--weights", default=None, help="HF safetensors checkpoint directory")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--parallel", default="auto",
                    help="auto | dp | reduce_tp | tp | tpK | per-stage layout, e.g. map:tp2,reduce:tp8")
    ap.add_argument("--max-model-len", type=int, default=None)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--batch-window-ms", type=float, default=5.0)
    ap.add_argument("--api-key", default=os.environ.get("MRSUM_SERVE_API_KEY"))
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=getattr(logging, a.log_level.upper()), format="%(asctime)s %(name)s %(message)s")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # before any HIP call (dmabuf IPC for RCCL)
    import torch
    from .engine.provider import LocalEngineProvider

    # ranks with no share of a batch wait in the stage all-gather for as long as the longest generation
    # runs (a 70B fp8 request near max_model_len, a big concurrent batch): give the collective watchdog
    # a serving-scale bound instead of the pipeline's 600 s (MRSUM_DIST_TIMEOUT still overrides)
    pdist.init_distributed_from_env(timeout_s=float(os.environ.get("MRSUM_DIST_TIMEOUT", "21600")))
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    provider = LocalEngineProvider(a.model, LLMConfig(), tp=a.tp, dtype=a.dtype, weights=a.weights,
                                   max_model_len=a.max_model_len, use_graphs=not a.no_graphs, parallel=a.parallel)
    provider.warm()
    batcher = make_batcher(provider, a.max_batch, a.batch_window_ms / 1000.0)
    if pdist.is_initialized() and provider.par.rank != 0:
        follower_loop(provider)
        pdist.shutdown()
        return 0
    import uvicorn
    batcher.start()
    app = build_app(batcher, a.served_model_name or a.model, a.api_key)
    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level=a.log_level.lower())
    finally:
        batcher.shutdown()
        pdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
