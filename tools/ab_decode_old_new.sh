set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 1,10,39 --ctx 4000 --new 256 | sed "s|^{|{\"tree\": \"$t\", |") || exit 1
  done
done
