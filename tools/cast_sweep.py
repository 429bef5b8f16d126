"""cast_sweep.py — occupancy caps for the fused-cast kernels (cast_segs_kernel), interleaved.

Runs tools/cast_probe.py in a fresh process per setting (the caps are read once per process):
TIPS_CAST_LDS_PACK / TIPS_CAST_LDS_UNPACK give each workgroup that many bytes of dynamic LDS,
so at most 160 KiB / (bytes + the kernel's own ~1 KiB) workgroups share a CU. Each round runs
every setting once, in a rotated order; one JSON line per run (the probe's gated device time per
config-5 round trip), then one summary line per setting (median over rounds).

usage: python3 tools/cast_sweep.py [rounds] [pack|unpack|tile|cast_tile|variant]
  (tile: TIPS_COPY_TILE_BYTES 4/8/16 KiB, before the cast had its own; cast_tile: TIPS_CAST_TILE_BYTES; variant: TIPS_CAST_VARIANT, load / store policies)
"""
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CAPS = {"none": 0, "7/CU": 22272, "6/CU": 26112, "5/CU": 31488, "4/CU": 39680, "3/CU": 53504}
TILES = {"4KiB": 4096, "8KiB": 8192, "16KiB": 16384}  # the cast layout's tile (wire bytes)
# TIPS_CAST_VARIANT: bit 0 plain loads (else nt), bits 1-2 the store (0 sc1, 1 plain, 2 nt)
VARIANTS = {"nt/sc1": 0, "plain/sc1": 1, "nt/plain": 2, "plain/plain": 3, "nt/nt": 4, "plain/nt": 5,
            "nt/sc1+lds16": 8}
if os.environ.get("CAST_SWEEP_VARIANTS"):  # e.g. "0,8": a subset
    VARIANTS = {k: v for k, v in VARIANTS.items() if str(v) in os.environ["CAST_SWEEP_VARIANTS"].split(",")}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    which = sys.argv[2] if len(sys.argv) > 2 else "pack"
    var = {"pack": "TIPS_CAST_LDS_PACK", "unpack": "TIPS_CAST_LDS_UNPACK", "tile": "TIPS_COPY_TILE_BYTES",
           "cast_tile": "TIPS_CAST_TILE_BYTES",
           "variant": "TIPS_CAST_VARIANT"}[which]
    CAPS = {"tile": TILES, "cast_tile": TILES, "variant": VARIANTS}.get(which, globals()["CAPS"])
    names = list(CAPS)
    res = {n: [] for n in names}
    for r in range(rounds):
        order = names[r % len(names):] + names[:r % len(names)]
        for n in order:
            env = dict(os.environ, **{var: str(CAPS[n])})
            p = subprocess.run([sys.executable, os.path.join(HERE, "cast_probe.py"), "40"]
                               + os.environ.get("CAST_PROBE_ARGS", "").split(), env=env,
                               capture_output=True, text=True, timeout=180)
            if p.returncode != 0:
                print(json.dumps({"cap": n, "error": p.stderr[-400:]}), flush=True)
                sys.exit(1)
            for line in p.stdout.splitlines():
                d = json.loads(line)
                if d.get("mode") == "gated":
                    res[n].append(d["us_per_call"])
                    print(json.dumps({"round": r, "dir": which, "cap": n, "lds": CAPS[n], "us": d["us_per_call"],
                                      "frac": d["frac"]}), flush=True)
    for n in names:
        m = statistics.median(res[n])
        print(json.dumps({"summary": which, "cap": n, "lds": CAPS[n], "us_median": m, "runs": res[n],
                          "probe_args": os.environ.get("CAST_PROBE_ARGS", "")}), flush=True)


if __name__ == "__main__":
    main()
