#!/usr/bin/env python3
"""Summarise a level trace (tools/bench_graph.py --trace-out) by level ranges: count, mean
frontier, total and per-level ms.   python tools/level_ranges.py trace.json [bucket]"""
import json
import sys

recs = json.load(open(sys.argv[1]))
bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 500
print(f"{len(recs)} levels, {sum(r['ms'] for r in recs):.2f} ms")
for b in range(0, len(recs), bucket):
    part = recs[b:b + bucket]
    ms = sum(r["ms"] for r in part)
    nf = sum(max(r["nf"], 0) for r in part) / len(part)
    print(f"levels {part[0]['level']}-{part[-1]['level']}: mean frontier {nf:.0f}, "
          f"{ms:.2f} ms, {1e3 * ms / len(part):.1f} us/level")
