# round 4: first check from codes (compressed min-sum) + ldpc_decode_codes
set -o pipefail
mkdir -p gpurun_out/ff
timeout -k 10 600 python -u -m pytest tests/test_coded_input.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "msa or coded or nonfinite or codes" > gpurun_out/ff/pytest.txt 2>&1 || exit 1
for ffp in 0 1 0 1; do
  timeout -k 10 200 python bench.py --algo msa --p 0.002 --batch-per-gpu 1000000 --secondary 0 --cpu-seconds 1 --steps 2 --warmup 1 --ffp $ffp > gpurun_out/ff/msa_ffp${ffp}_$RANDOM.json 2>>gpurun_out/ff/bench.err || exit 1
done
LDPC_API_TIMING=1 timeout -k 10 200 python bench.py --workload dna272 --steps 3 > gpurun_out/ff/dna272.json 2> gpurun_out/ff/dna272.err
