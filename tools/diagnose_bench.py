#!/usr/bin/env python3
"""Read a bench.py JSON line (a file holding it -- BENCH_rNN.json, a gpurun log -- or stdin) and say what a
multi-GPU run's numbers mean, in the order to look at them: did every rank run and was the timed work pinned,
did the P2P paths pass their self-test and stay up (recoveries), how far each stage's measured seconds are
from the planner's prediction at the layout it ran, and the cross-GPU all-reduce latency per TP degree that
the planner's choice depends on (re-plan with it: tools/plan_stages.py --ar-lat-us).

    python tools/diagnose_bench.py BENCH_r06.json
    python bench.py ... | python tools/diagnose_bench.py -

Prints one finding per line ("ok: ..." / "CHECK: ..."); exit code 0 either way (a reading aid, not a gate).
"""
import json
import sys

SLOW = 1.3        # measured / predicted above this: the stage ran slower than the planner's model of it
PUSH_HIGH_US = 20.0  # cross-GPU push all-reduce latency the round-6 planner assumed at most (ar_lat_us 5-20)


def bench_lines(text):
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            try:
                yield json.loads(line)
            except ValueError:
                continue


def diagnose(d):
    out = []
    n = d.get("n_gpus", 1)
    seen = d.get("ranks_seen")
    out.append(("ok" if seen in (None, n) else "CHECK") + ": ranks seen %s of %s (backend %s)" % (seen, n, d.get("backend")))
    tw = d.get("timed_work") or {}
    if tw:
        good = tw.get("pinned_ok") and not tw.get("errors")
        out.append(("ok" if good else "CHECK") + ": timed work %s requests, %s errors, %s of %s tokens, pinned_ok %s"
                   % (tw.get("requests"), tw.get("errors"), tw.get("completion_tokens"), tw.get("requested_tokens"),
                      tw.get("pinned_ok")))
    for deg, st in sorted((d.get("p2p_selftest") or {}).items()):
        if not isinstance(st, dict):  # e.g. "off (RCCL)": the TP engine runs its all-reduces on RCCL
            out.append("ok: P2P self-test %s: %s" % (deg, st))
            continue
        bad = sorted(k for k, v in st.items() if v in ("failed", "untested"))
        why = st.get("why") or {}
        msg = (" failed: " + ", ".join("%s (%s)" % (k, why.get(k, "?")) for k in bad)) if bad else " every exercised path ok"
        if st.get("unusable"):
            bad.append("unusable")
            msg += "; handle unusable: " + st["unusable"]
        out.append(("CHECK" if bad else "ok") + ": P2P self-test %s%s" % (deg, msg))
    rec = d.get("ar_recoveries") or 0
    out.append(("CHECK" if rec else "ok") + ": custom all-reduce recoveries %d" % rec)
    for name, s in (d.get("stages") or {}).items():
        p, m = s.get("predicted_s"), s.get("measured_s")
        if not p or m is None:
            out.append("CHECK: stage %s tp %s has no prediction (measured %s s)" % (name, s.get("tp"), m))
            continue
        r = m / p
        out.append(("CHECK" if r > SLOW else "ok") + ": stage %s at tp %s: measured %.3f s vs predicted %.3f s (x%.2f)%s"
                   % (name, s.get("tp"), m, p, r,
                      "; compare the tp%s push latency below with the planner's ar_lat" % s.get("tp") if r > SLOW else ""))
    for deg, lat in sorted((d.get("p2p_latency_us") or {}).items()):
        if not isinstance(lat, dict) or "error" in lat:
            out.append("CHECK: P2P latency probe %s: %s" % (deg, lat))
            continue
        push = lat.get("push_us", lat.get("fused_us"))
        out.append(("CHECK" if push is not None and push > PUSH_HIGH_US else "ok")
                   + ": %s decode all-reduce cross-GPU cost %s us + %s us/row (push), fused %s us -- re-plan with "
                   "tools/plan_stages.py --worlds %s --ar-lat-us %s" % (deg, push, lat.get("push_us_per_row"),
                                                                       lat.get("fused_us"), n, push))
    return out


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "-"
    text = sys.stdin.read() if src == "-" else open(src).read()
    found = False
    for d in bench_lines(text):
        found = True
        print("# %s: %s %s (n_gpus %s, %s)" % (d.get("metric"), d.get("value"), d.get("unit"), d.get("n_gpus"),
                                               (d.get("config") or {}).get("parallelism")))
        for line in diagnose(d):
            print(line)
    if not found:
        print("no bench.py JSON line found in %s" % src)


if __name__ == "__main__":
    main()
