#!/bin/bash
# round-3 session: GEMV lab, then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r03s1
timeout -k 10 120 ./tools/lab_gemv > gpurun_out/r03s1/lab_gemv.txt 2>&1 || { echo "lab failed"; tail gpurun_out/r03s1/lab_gemv.txt; exit 1; }
cat gpurun_out/r03s1/lab_gemv.txt
bash tools/gpu_tests.sh r03s1 tests 0 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s1/smoke.log 2>&1 || { tail -20 gpurun_out/r03s1/smoke.log; exit 1; }
tail -3 gpurun_out/r03s1/smoke.log
