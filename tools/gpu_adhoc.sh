set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r1m; mkdir -p $OUT; cd $R
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python tools/sweep.py --batch 65536 --chunk 16384 --rounds 1 --algo msa --p 0.002 --configs 3:1:0:0:1 > $OUT/sweep_msa.jsonl 2>$OUT/sweep_msa.err; rc=$?; echo "sweep msa rc=$rc"; cat $OUT/sweep_msa.jsonl; tail -3 $OUT/sweep_msa.err
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --steps 1 --warmup 0 --cpu-seconds 8 > $OUT/msa_1m.json 2> $OUT/msa_1m.err; rc=$?; echo "msa 1M rc=$rc"; cat $OUT/msa_1m.json; tail -3 $OUT/msa_1m.err
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; rc=$?; echo "default rc=$rc"; cat $OUT/bench_default.json; tail -3 $OUT/bench_default.err
