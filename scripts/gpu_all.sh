#!/bin/bash
# One box, everything: the full GPU check (tests, smoke, bench, kernel stats) then the rank-count
# sweep and the PMC passes.  Each step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_full.sh && bash scripts/gpu_scale_and_pmc.sh
