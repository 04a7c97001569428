"""The key numbers of a final evidence set (tools/r06_final.sh) in one table.

    python tools/final_summary.py [profiles/r06final_]
"""
import json
import os
import sys


def line(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def main(prefix):
    def p(name):
        return prefix + name

    out = []
    for i in (1, 2, 3):
        f = p(f"driver_cmd_bench_{i}.json")
        if os.path.exists(f):
            d = line(f)
            r = d["roofline"]
            out.append(f"driver command {i}: {d['value']:8.1f} GiB/s  ms/step {d['ms_per_step']:.4f}  "
                       f"scan frac {r['frac']:.3f}  pass {r['pipeline_avg_ms']:.4f} ms")
    for wl in ("c1", "c2", "c3", "c4", "c4f", "c4b", "c4b_2", "c4bl", "n2_rehearsal", "rccl_one_rank"):
        f = p(f"bench_{wl}.json")
        if not os.path.exists(f):
            continue
        d = line(f)
        r = d.get("roofline", {})
        s = f"{wl:14s} {d['value']:8.2f} GiB/s"
        if r.get("bound") == "hbm" and "pipeline_avg_ms" in r:
            s += f"  scan frac {r['frac']:.3f}  scan {r['kernel_avg_ms']:.4f} ms  pass {r['pipeline_avg_ms']:.4f} ms"
        if "wall_set_by" in r:
            s += f"  wall: {r['wall_set_by']} ({r.get('named_over_wall')})"
        cb = d.get("cpu_baseline") or {}
        if cb.get("value"):
            s += f"  cpu {cb['value']:.2f} ({cb.get('cores')} core)"
            if cb.get("multi_thread"):
                s += f", {cb['multi_thread']['value']} ({cb['multi_thread']['cores']})"
        cd = d.get("chunk_digests")
        if cd:
            s += (f"\n{'':14s} digests {cd['value']} / hybrid {cd['hybrid']['value']} / "
                  f"pipelined {cd['pipelined_with_chunking']['value']} GiB/s")
        en = d.get("encode")
        if en:
            s += f"\n{'':14s} encode {en['value']} GiB/s ({en['ms_per_pass']} ms/pass)"
        e2e = d.get("e2e_host_path")
        if e2e:
            s += f"\n{'':14s} host path {e2e['value']} pageable / {e2e['pinned']['value']} pinned GiB/s"
        out.append(s)
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join("profiles", "r06final_"))
