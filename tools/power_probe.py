"""GPU power and clocks over the driver's bench window: a sampler thread reads
amdsmi (socket power, gfx clock, throttle status from the GPU metrics table)
as fast as it can while the main thread runs `--warmup` + `--steps` pipelined
passes (two streams, as bench.py) and then 20 single-stream passes.  Prints a
timeline in 1-ms bins with the pass boundaries.

    python tools/power_probe.py [--steps 20 --warmup 5 --streams 2] [--walk]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--tail", type=int, default=20)
    args = ap.parse_args()
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    try:
        cap = amdsmi.amdsmi_get_power_cap_info(h)
    except Exception as e:  # noqa: BLE001
        cap = repr(e)
    samples = []
    stop = [False]

    def sampler():
        while not stop[0]:
            t = time.perf_counter()
            rec = [t]
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                rec += [m.get("current_socket_power"), m.get("average_socket_power"), m.get("current_gfxclk"),
                        m.get("average_gfxclk_frequency"), m.get("throttle_status"), m.get("indep_throttle_status"),
                        m.get("temperature_hotspot")]
            except Exception as e:  # noqa: BLE001
                rec += [repr(e)]
            samples.append(rec)

    import torch
    from bench import WORKLOADS, make_buffers
    from plakar_amd import _lib, chunkers, device
    _lib.ensure_init()
    dev = torch.device("cuda", 0)
    wl = WORKLOADS["c1"]
    bufs = make_buffers(torch, wl, 0, dev, wl["size"])
    opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
    batches = [device.DeviceBatch(bufs, opts, final=True) for _ in range(args.streams)]
    streams = [torch.cuda.Stream(dev) for _ in range(args.streams)]
    torch.cuda.synchronize()
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    time.sleep(0.02)
    marks = []
    t0 = time.perf_counter()
    for i in range(args.warmup):
        batches[i % args.streams].launch(streams[i % args.streams])
    torch.cuda.synchronize()
    marks.append(("timed start", time.perf_counter()))
    for i in range(args.steps):
        batches[i % args.streams].launch(streams[i % args.streams])
    torch.cuda.synchronize()
    marks.append(("timed end", time.perf_counter()))
    for i in range(args.tail):
        batches[0].launch(streams[0])
    torch.cuda.synchronize()
    marks.append(("tail end", time.perf_counter()))
    time.sleep(0.02)
    stop[0] = True
    th.join()
    print(f"power cap info: {cap}")
    print(f"{len(samples)} samples; marks: " + ", ".join(f"{n} {1e3 * (t - t0):.2f} ms" for n, t in marks))
    print("t_ms   cur_W avg_W gfxclk avg_gfxclk throttle indep_throttle hotspot_C")
    for r in samples:
        if len(r) > 2:
            print(f"{1e3 * (r[0] - t0):7.2f} " + " ".join(str(x) for x in r[1:]))
        else:
            print(f"{1e3 * (r[0] - t0):7.2f} {r[1]}")
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
