set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r1p; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 600 python -m pytest tests/test_cli_gpu.py -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch-per-gpu 8192 > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err; rc=$?; echo "2-rank rc=$rc"; cat $OUT/bench_2rank.json; tail -5 $OUT/bench_2rank.err
