#!/bin/bash
# Same-box decode-step A/B: .ab_old (a git worktree of an earlier commit, built in-tree) vs this tree,
# alternating twice (tools/bench_decode.py B=1/10/39 at 4k context).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches ${BATCHES:-1,10,39} --ctx 4000 --new 256 | sed "s|^{|{\"tree\": \"$t\", |") || exit 1
  done
done
