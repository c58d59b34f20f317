#!/usr/bin/env python3
"""Markdown table of tools/burst_sizes.py output (one JSON object a line):
per burst size, the median call time of decode (RX) and encode (TX) from
pinned and from pageable memory, datagrams/s of the pinned RX call, and the
oracle's time for the same call on 1 and 16 threads.

  python tools/burst_sizes_table.py profiles/round6/burst_sizes.jsonl
"""
import json
import sys


def main(path):
    rows = {}
    for ln in open(path):
        if not ln.startswith("{"):
            continue
        r = json.loads(ln)
        rows.setdefault(r["n"], {})[(r["kind"], r["memory"])] = r
    print("| datagrams | RX pinned µs | RX pageable µs | TX pinned µs | TX pageable µs "
          "| RX pinned M/s | oracle RX 1 thread µs | oracle RX 16 threads µs "
          "| GPU / 1 core |")
    print("|---|---|---|---|---|---|---|---|---|")
    for n in sorted(rows):
        g = rows[n]

        def med(k, m):
            return g.get((k, m), {}).get("median_us")
        rx = g.get(("rx", "pinned"), {})
        o1, o16 = rx.get("oracle_1t_us"), rx.get("oracle_16t_us")
        ratio = f"{o1 / rx['median_us']:.1f}x" if o1 and rx.get("median_us") else "—"

        def f(v):
            return "—" if v is None else (f"{v:,.1f}" if v < 1000 else f"{v:,.0f}")
        print(f"| {n:,} | {f(med('rx', 'pinned'))} | {f(med('rx', 'pageable'))} "
              f"| {f(med('tx', 'pinned'))} | {f(med('tx', 'pageable'))} "
              f"| {rx.get('datagrams_per_s', 0) / 1e6:.2f} | {f(o1)} | {f(o16)} | {ratio} |")


if __name__ == "__main__":
    main(sys.argv[1])
