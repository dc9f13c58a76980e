#!/bin/bash
# full GPU suite + smoke on the current tree, then configs[4] (pipeline) and offline SortFormer benches
set -o pipefail
T=gpurun_out/r03k; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > $T/pytest.log 2>&1; rc=$?
tail -3 $T/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $T/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -4 $T/smoke.log
timeout -k 10 600 python tools/pipeline_bench.py --no-cpu --mode sequential > $T/pipeline.json 2> $T/pipeline.err || { tail -5 $T/pipeline.err; exit 1; }
cut -c1-600 $T/pipeline.json
timeout -k 10 300 python tools/sf_bench.py --cpu-seconds 0 > $T/sf_bench.json 2> $T/sf_bench.err || { tail -5 $T/sf_bench.err; exit 1; }
cut -c1-600 $T/sf_bench.json
