"""cast_probe.py — where the time of Compression.fp16's fused round trip goes (config 5, one rank).

bench.py's config5_resnet50.fp16_compressed host-times tips_amd._reduce_grads(grads,
compression=Compression.fp16) over 4 rotating gradient sets: cast pack (f32 -> f16 into the
buckets), the wire-type allreduce (the identity at one rank) and the cast unpack (f16 -> f32 into
one flat output). This probe times the same call three ways, one JSON line each:
  host      wall time per call, back to back (what bench.py reports)
  events    HIP events around the same calls on torch's stream (the device's span)
  gated     the calls queued behind a spin kernel, so the device runs them back to back without
            waiting for the host: the device-side cost alone
Run it under `rocprofv3 --kernel-trace --stats` to split the device span per kernel.

usage: python3 tools/cast_probe.py [steps] [--config4]   (--config4: config 4's 1000 gradients instead;
       the host lines then also give tips_fusion_stats' deltas and the fp32 allreduce_grads body's time)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 40
    config4 = "--config4" in sys.argv
    import torch

    import bench
    import tips_amd
    torch.cuda.set_device(0)
    tips_amd.init()
    sizes = bench.fused1000_sizes() if config4 else bench.resnet50_grad_sizes()
    rot = 4
    gens = [torch.Generator(device="cuda").manual_seed(5000 + k) for k in range(rot)]
    grads = [[torch.rand(n, device="cuda", generator=gens[k]) + 0.5 for n in sizes] for k in range(rot)]
    fp16 = tips_amd.Compression.fp16
    elems = sum(sizes)
    moved = 12 * elems  # pack: 4 B read + 2 B written; unpack: 2 B read + 4 B written
    call = lambda i: tips_amd._reduce_grads(grads[i % rot], compression=fp16)  # noqa: E731
    keep = []
    for i in range(2 * rot):
        keep.append(call(i))
    torch.cuda.synchronize()
    keep.clear()

    def line(mode, us):
        print(json.dumps({"mode": mode, "us_per_call": round(us, 2), "algorithmic_bytes": moved,
                          "GBps": round(moved / us / 1e3, 1), "frac": round(moved / us / 1e3 / 8000.0, 4)}), flush=True)

    st0 = tips_amd.fusion_stats()
    t0 = time.perf_counter()
    for i in range(steps):
        call(i)
    torch.cuda.synchronize()
    line("host", (time.perf_counter() - t0) * 1e6 / steps)
    if config4:
        print(json.dumps({"fusion_stats_before": st0, "after": tips_amd.fusion_stats()}), flush=True)
        for name, fn in (("fp32_reduce_grads", lambda i: tips_amd._reduce_grads(grads[i % rot])),):
            try:
                for i in range(rot):
                    fn(i)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    fn(i)
                torch.cuda.synchronize()
                print(json.dumps({"mode": "host", "call": name, "us_per_call": round((time.perf_counter() - t0) * 1e6 / steps, 2)}), flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"call": name, "error": str(e)}), flush=True)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for i in range(steps):
            call(i)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(12)

    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(steps):
        call(i)
    e1.record(s)
    torch.cuda.synchronize()
    line("events", e0.elapsed_time(e1) * 1e3 / steps)

    torch.cuda._sleep(50_000_000)
    e0.record(s)
    for i in range(steps):
        call(i)
    e1.record(s)
    torch.cuda.synchronize()
    line("gated", e0.elapsed_time(e1) * 1e3 / steps)
    got = call(0)
    torch.cuda.synchronize()
    ref = torch.cat([g.reshape(-1) for g in grads[0]]).half().float()
    ok = torch.equal(torch.cat([g.reshape(-1) for g in got]), ref)
    print(json.dumps({"check": "round trip through f16, bit-exact" if ok else "FAIL"}), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
