#!/bin/bash
# After the narrow K(W, W): 1-GPU bench, inner-phase probe at 60k / 1M, 60k kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/r4ww_bench1.json > gpurun_out/r4ww_bench1.log 2>&1 \
  || { tail -20 gpurun_out/r4ww_bench1.log; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r4ww_bench1.json"))
print("1 GPU", a["value"], a["iterations"], a["b"], a["n_sv"], a["accuracy"], a.get("f64_input_fit_ms"), a["pairwise_solver"]["fit_ms"], a["timings_ms"])
PY
rm -f gpurun_out/r4ww_prof.txt
for n in 60000 1000000; do
  SVM355_DECOMP_PROF=1 timeout -k 10 200 python -u scripts/decomp_inner_probe.py $n 1024 >> gpurun_out/r4ww_prof.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r4ww_prof.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4wwprof -o run -- \
  python3 bench.py --steps 10 --warmup 3 --decomp-fits 0 --f64-fits 0 > gpurun_out/r4wwprof.log 2>&1 || { tail -5 gpurun_out/r4wwprof.log; exit 1; }
