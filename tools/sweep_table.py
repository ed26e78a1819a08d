"""Table of a ceiling_sweep.py JSONL (development tool): one row per shape with % of
8 TB/s for the rule, tuned, read+write ceiling, and the tuned order.
usage: python tools/sweep_table.py file.jsonl [...]"""
import json
import sys

for path in sys.argv[1:]:
    for ln in open(path):
        if not ln.startswith("{"):
            continue
        r = json.loads(ln)
        if "skipped" in r:
            print(f"{r['shape']}: skipped ({r['skipped']})")
            continue
        p = r["pct_of_8TBs"]
        print(f"{r['k']:>3},{r['m']:<2} S={r['S']:>10} {r['erase']:>9} {r['layout']:>22} "
              f"prod {p.get('prod', 0):6.2f} tuned {p.get('tuned', 0):6.2f} "
              f"r+w {p.get('read+write', 0):6.2f} {r.get('tuned_orders')}")
