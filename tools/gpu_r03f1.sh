#!/bin/bash
# round-3 final, part 1: logits-kernel A/B (turbo), then the full GPU suite and smoke()
set -o pipefail
bash tools/gpu_ab.sh ablg2 OWK_LOGITS_REG=0 OWK_LOGITS_REG=1 --steps 2 --warmup 1 --model large-v3-turbo || exit $?
T=gpurun_out/r03f1; mkdir -p $T
export OWK_MODEL_CACHE=/tmp/owk_models
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > $T/pytest.log 2>&1; rc=$?
tail -3 $T/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $T/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { tail -20 $T/smoke.log; exit 1; }
tail -4 $T/smoke.log
