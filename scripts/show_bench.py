#!/usr/bin/env python3
"""Print the headline and the named legs of a bench.py JSON line: show_bench.py FILE [leg ...]"""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "kernels", json.dumps(d.get("kernels")))
for leg in sys.argv[2:]:
    if leg in d:
        v = d[leg]
        print(leg, json.dumps({k: v[k] for k in v if not isinstance(v[k], (dict, list))}))
