#!/bin/bash
# Round-2 first GPU session: the whole -m gpu suite and smoke on HEAD, the
# default bench line, and a fresh-engine A/B of the ping-pong resident
# schedule against the default resident pool.  Each GPU step has its own
# limit; a failing step ends the session.
set -u
TAG=${1:-r2a}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; tail -c 1500 "$OUT/$name.out"; tail -3 "$OUT/$name.err"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
run ab_pingpong 300 python -u tools/ab_engines.py --fresh 4 --var res: --var pp:LDPC_PINGPONG=1
exit 0
