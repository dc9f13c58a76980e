#!/bin/bash
set -o pipefail
for nt in 0 2 4; do OWK_ROWS_NT=$nt timeout -k 10 120 python tools/logits_gemm_bench.py || exit 1; done
