# Sweep LDPC_VAR_CPW (BP variable phase columns per wave) on the default
# bench workload; interleaved repeats to see run-to-run noise.
set -o pipefail
mkdir -p gpurun_out/cpw
for rep in 1 2; do
for c in ${CPWS:-1 8}; do
  LDPC_VAR_CPW=$c timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 3 --warmup 1 > gpurun_out/cpw/bench_${c}_$rep.json 2> gpurun_out/cpw/bench_${c}_$rep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/cpw/bench_${c}_$rep.json'));r=d['roofline'];print($c, $rep, d['value'], r['avg_ms']['check'], r['avg_ms']['variable'])"
done
done
