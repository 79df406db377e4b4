set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r1o; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 0 --cpu-seconds 8 > $OUT/msa_1m.json 2> $OUT/msa_1m.err; rc=$?; echo "msa 1M rc=$rc"; cat $OUT/msa_1m.json; tail -3 $OUT/msa_1m.err
