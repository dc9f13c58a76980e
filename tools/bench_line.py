"""One-line summary of a bench.py JSON output file: value, ms/step, token parity."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], (d.get("parity") or {}).get("tokens_equal"))
