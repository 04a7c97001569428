"""Per-pass timeline of a bench.py run from a rocprofv3 kernel-trace CSV.

    python tools/timeline.py <run_kernel_trace.csv> --warmup W --steps K [--first-kernel k_scan]

A pass starts at a scan launch (k_scan / k_scan_f).  The bench does W warm-up
passes, then K timed ones; this prints, for every pass of the first W + K,
its scan duration, the start-to-start gap to the next pass, and the span of
the timed region (first timed scan start -> last kernel end of pass W+K-1),
which is what bench.py's wall clock measures minus host launch latency.
"""
import argparse
import csv
from collections import defaultdict


def load(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--bins", type=int, default=0, help="only print per-bin pass rates (bins of this many passes)")
    a = ap.parse_args()
    ks = load(a.csv)
    is_scan = lambda n: n.endswith("k_scan") or n.endswith("k_scan_f")  # noqa: E731
    starts = [i for i, (_, _, n) in enumerate(ks) if is_scan(n)]
    npass = a.warmup + a.steps
    if len(starts) < npass:
        raise SystemExit(f"only {len(starts)} scans in the trace")
    if a.bins:
        t = [ks[i][0] for i in starts[:npass + 1]]
        print("passes        us/pass   scan_us(avg)   resolve_us(avg)")
        for b0 in range(0, npass, a.bins):
            b1 = min(npass, b0 + a.bins)
            if b1 >= len(t):
                break
            sc = [(ks[starts[p]][1] - ks[starts[p]][0]) / 1e3 for p in range(b0, b1)]
            rs = [(e - s) / 1e3 for s, e, n in ks[starts[b0]:starts[b1]] if n.endswith("k_resolve")]
            print(f"{b0:5d}-{b1 - 1:<5d} {(t[b1] - t[b0]) / 1e3 / (b1 - b0):9.1f} {sum(sc) / len(sc):12.1f} "
                  f"{(sum(rs) / len(rs)) if rs else 0:14.1f}")
        return
    print(f"{'pass':>4} {'t0_us':>10} {'scan_us':>8} {'gap_next_us':>11}  kernels (us)")
    per = defaultdict(list)
    for p in range(npass):
        i0 = starts[p]
        i1 = starts[p + 1] if p + 1 < len(starts) else len(ks)
        s0 = ks[i0][0]
        nxt = ks[i1][0] - s0 if p + 1 < len(starts) else 0
        body = ks[i0:i1]
        desc = " ".join(f"{n.split('::')[-1]}={(e - s) / 1e3:.1f}" for s, e, n in body[:8])
        tag = "W" if p < a.warmup else "T"
        print(f"{tag}{p:>3} {(s0 - ks[starts[0]][0]) / 1e3:10.1f} {(ks[i0][1] - s0) / 1e3:8.1f} {nxt / 1e3:11.1f}  {desc}")
        if p >= a.warmup:
            for s, e, n in body:
                per[n.split("::")[-1]].append((e - s) / 1e3)
    t_first = ks[starts[a.warmup]][0]
    last = starts[npass] if npass < len(starts) else len(ks)
    # last kernel end among the timed passes (the two streams interleave, so take the max)
    t_end = max(e for s, e, n in ks[starts[a.warmup]:last])
    span = (t_end - t_first) / 1e3
    print(f"\ntimed region on the device: {span:.1f} us for {a.steps} passes = {span / a.steps:.1f} us/pass")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:16s} n={len(v):4d} avg={sum(v) / len(v):8.2f} min={min(v):8.2f} max={max(v):8.2f}")
    # bench.py's roofline loop: the next max(5, min(K, 50)) passes, one stream,
    # the scan alone on the device (its roofline.kernel_avg_ms)
    rsteps = max(5, min(a.steps, 50))
    roof = [(ks[i][1] - ks[i][0]) / 1e3 for i in starts[npass:npass + rsteps]]
    if len(roof) == rsteps:
        print(f"\nroofline loop (passes {npass}-{npass + rsteps - 1}, one stream): scan avg {sum(roof) / len(roof):.2f} us "
              f"min {min(roof):.2f} max {max(roof):.2f}")


if __name__ == "__main__":
    main()
