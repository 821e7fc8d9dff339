#!/usr/bin/env python3
"""Serving benchmark: the OpenAI-compatible server (serve.py) in-process on 127.0.0.1 over the local
engine; N clients send chat requests with Poisson arrivals (--rate req/s, 0 = all at once) of synthetic
transcript-chunk prompts and pinned completion lengths.  One JSON line: request / output-token throughput
and end-to-end latency percentiles (p50 / p90 / p99), plus the server's batching stats.

    python tools/bench_serve.py [--model llama3-8b] [--requests 64] [--rate 8] [--prompt-tokens 2000] [--new 256]
"""
import argparse
import json
import os
import random
import socket
import sys
import threading
import time
import urllib.request
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--rate", type=float, default=8.0, help="Poisson arrival rate (req/s); 0 = all at once")
    ap.add_argument("--prompt-tokens", type=int, default=2000)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=64)
    a = ap.parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import uvicorn
    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.serve import build_app, make_batcher
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript

    prov = LocalEngineProvider(a.model, LLMConfig(), dtype=a.dtype, ignore_eos=True, max_model_len=8192)
    prov.warm(capture_batch=a.max_batch)
    batcher = make_batcher(prov, a.max_batch, 0.005)
    batcher.start()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(build_app(batcher, a.model), host="127.0.0.1", port=port,
                                        log_level="warning", limit_concurrency=4 * a.requests))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    while not srv.started:
        time.sleep(0.05)

    # prompts: consecutive synthetic transcript text cut to ~prompt_tokens tokens each
    hours = max(1.0, a.requests * a.prompt_tokens / 14000)
    text = " ".join(seg["text"] for seg in synthetic_transcript(hours, seed=5)["segments"])
    ids = prov.tokenizer.encode_ordinary(text)
    prompts = [prov.tokenizer.decode(ids[i * a.prompt_tokens:(i + 1) * a.prompt_tokens]) for i in range(a.requests)]
    rng = random.Random(0)
    arrivals, t = [], 0.0
    for _ in range(a.requests):
        arrivals.append(t)
        t += rng.expovariate(a.rate) if a.rate > 0 else 0.0
    url = "http://127.0.0.1:%d/v1/chat/completions" % port

    def one(i):
        body = {"model": a.model, "messages": [{"role": "system", "content": "Summarize the transcript segment."},
                                               {"role": "user", "content": prompts[i]}],
                "max_tokens": a.new, "temperature": 0.3}
        wait = t0 + arrivals[i] - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        s = time.perf_counter()
        req = urllib.request.Request(url, data=json.dumps(body).encode(), headers={"Content-Type": "application/json"})
        out = json.loads(urllib.request.urlopen(req, timeout=600).read())
        return time.perf_counter() - s, out["usage"]["completion_tokens"], out["usage"]["prompt_tokens"]

    # warm-up request (first prefill / graph replay paths)
    t0 = time.perf_counter()
    arrivals_saved, arrivals = arrivals, [0.0] * a.requests
    one(0)
    arrivals = arrivals_saved
    t0 = time.perf_counter()
    with ThreadPoolExecutor(a.requests) as ex:
        res = list(ex.map(one, range(a.requests)))
    wall = time.perf_counter() - t0
    lat = sorted(r[0] for r in res)
    pct = lambda q: lat[min(len(lat) - 1, int(q * len(lat)))]  # noqa: E731
    out_tok = sum(r[1] for r in res)
    print(json.dumps({"metric": "serving throughput (OpenAI-compatible HTTP, continuous batching)", "model": a.model,
                      "dtype": a.dtype, "requests": a.requests, "rate_req_s": a.rate,
                      "prompt_tokens_mean": round(sum(r[2] for r in res) / len(res)), "new_tokens": a.new,
                      "wall_s": round(wall, 3), "req_per_s": round(a.requests / wall, 3),
                      "output_tok_per_s": round(out_tok / wall, 1),
                      "latency_s": {"p50": round(pct(0.5), 3), "p90": round(pct(0.9), 3), "p99": round(pct(0.99), 3)},
                      "server": batcher.stats, "engine_fed_requests": prov.engine.stats.get("fed_requests", 0),
                      "data": "synthetic transcript prompts; random-init weights; completions pinned to --new"}),
          flush=True)
    srv.should_exit = True
    th.join(10)
    batcher.shutdown(30)


if __name__ == "__main__":
    main()
