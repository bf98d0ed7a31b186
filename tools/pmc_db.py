"""Per-dispatch PMC counters from a rocprofv3 sqlite output (measurement tool).

    python tools/pmc_db.py gpurun_out/pmc_emit_TAG [kernel-substring]
"""
import collections
import glob
import json
import sqlite3
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for db in sorted(glob.glob(f"{d}/**/*.db", recursive=True)):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info('counters_collection')")]
    rows = collections.defaultdict(dict)
    for r in c.execute("select * from counters_collection"):
        r = dict(zip(cols, r))
        if sub in r["kernel_name"]:
            rows[(r["dispatch_id"], r["kernel_name"])][r["counter_name"]] = r["value"]
    for (disp, name), v in sorted(rows.items()):
        print(json.dumps({"dispatch": disp, "kernel": name[:60],
                          **{k: int(x) for k, x in sorted(v.items())}}))
