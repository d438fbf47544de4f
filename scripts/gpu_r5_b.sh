#!/bin/bash
# Round 5: (1) where the cold decomposition fit's extra time goes (HIP API + kernel trace of a fresh
# process: device init, cold fit, two warm fits); (2) the two SIGSEGVs of round 4, re-run under the
# same profiler with the crash-evidence handler (signal, PC, backtrace, /proc/self/maps to a file):
#   - the exit-time crash of a profiled single-GPU fit (r4wprof.log)
#   - the 8-thread-rank 1M loopback rehearsal under --kernel-trace (r4d1m.log)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp
export SVM355_CRASH_MAPS=$PWD/gpurun_out/r5b/crash_{pid}.txt
cd /tmp
timeout -k 10 240 rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5b/cold -o run \
  -- python3 $GRAFT_REPO_ROOT/scripts/cold_fit_decomp_probe.py 60000 > $GRAFT_REPO_ROOT/gpurun_out/r5b/cold.log 2>&1
echo "cold probe under rocprofv3: rc $?"
grep -E "^fit|^device" $GRAFT_REPO_ROOT/gpurun_out/r5b/cold.log
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 scripts/cold_fit_decomp_probe.py 60000 > gpurun_out/r5b/cold_noprof.log 2>&1
echo "cold probe without profiler: rc $?"
grep -E "^fit|^device" gpurun_out/r5b/cold_noprof.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5b/d1m -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 8 --transport loopback --parallel decomp --rows 1000000 --test-rows 2000 \
  --steps 1 --warmup 1 --cascade-steps 0 --baseline-1gpu 1 --out $GRAFT_REPO_ROOT/gpurun_out/r5b/d1m.json \
  > $GRAFT_REPO_ROOT/gpurun_out/r5b/d1m.log 2>&1
echo "1M P=8 loopback rehearsal under rocprofv3: rc $?"
tail -c 600 $GRAFT_REPO_ROOT/gpurun_out/r5b/d1m.log
ls $GRAFT_REPO_ROOT/gpurun_out/r5b/
exit 0
