set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r1i; mkdir -p $OUT; cd $R
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python tools/sweep.py --batch 16384 --rounds 2 --configs 3:1:0:0:0,3:1:0:0:1 > $OUT/sweep_bp.jsonl 2>$OUT/sweep_bp.err; echo "sweep bp rc=$?"; cat $OUT/sweep_bp.jsonl; tail -3 $OUT/sweep_bp.err
timeout -k 10 600 python tools/sweep.py --batch 16384 --rounds 2 --algo msa --p 0.002 --configs 3:1:0:0:0,3:1:0:0:1 > $OUT/sweep_msa.jsonl 2>$OUT/sweep_msa.err; echo "sweep msa rc=$?"; cat $OUT/sweep_msa.jsonl; tail -3 $OUT/sweep_msa.err
timeout -k 10 600 python tools/sweep.py --batch 16384 --rounds 2 --p 0.002 --configs 3:1:0:0:0,3:1:0:0:1 > $OUT/sweep_bp2.jsonl 2>$OUT/sweep_bp2.err; echo "sweep bp p.002 rc=$?"; cat $OUT/sweep_bp2.jsonl; tail -3 $OUT/sweep_bp2.err
