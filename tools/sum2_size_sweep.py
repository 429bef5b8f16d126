"""The 2-input sum's HBM rate against operand size and launch shape (the p = 2
fold of 2 x 128 MiB ran at 0.75 of HBM against 0.82 for config 2's 2 x 256 MiB).

For each operand size, every variant (tips_sum_variant, the development library) runs over 4
rotating buffer sets (so no launch finds its operands in the Infinity Cache), interleaved over
ROUNDS rounds; one JSON line per (size, variant) with the best round's us per launch and its
fraction of 8 TB/s (3 x size bytes per launch). VARIANT_SET=policy sweeps cache policies instead of
launch shapes, VARIANT_SET=map workgroup -> tile maps."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tips_amd import _lib  # noqa: E402

D = _lib.dev()
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
SIZES = [int(x) for x in os.environ.get("SIZES_MIB", "64,128,192,256").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", "3"))
# (name, mode, unroll, nt index, LDS bytes per workgroup, threads): mode 3 = buffer ops (nt index 1 =
# nt loads + sc1 stores, the shipped policy); blocks = unused LDS reserved per workgroup
VARIANTS = [("shipped", 3, 1, 1, 0, 256), ("u2", 3, 2, 1, 0, 256), ("u4", 3, 4, 1, 0, 256),
            ("t512", 3, 1, 1, 0, 512), ("t128", 3, 1, 1, 0, 128), ("u2t512", 3, 2, 1, 0, 512),
            ("cap8", 3, 1, 1, 20480, 256), ("cap4", 3, 1, 1, 40960, 256), ("cap3", 3, 1, 1, 53248, 256)]
if os.environ.get("VARIANT_SET") == "policy":
    # cache policies (nt index into the (load aux, store aux) pairs of sum2_dispatch's mode 3):
    # does the best store / load policy depend on the operand size?
    VARIANTS = [("shipped", 3, 1, 1, 0, 256), ("st_plain", 3, 1, 0, 0, 256), ("st_nt", 3, 1, 7, 0, 256),
                ("st_sc1glc", 3, 1, 2, 0, 256), ("st_ntsc1", 3, 1, 10, 0, 256), ("st_sc0ntsc1", 3, 1, 11, 0, 256),
                ("st_sc0", 3, 1, 12, 0, 256), ("st_sc0nt", 3, 1, 13, 0, 256), ("ld_plain", 3, 1, 8, 0, 256),
                ("ld_nt2_st_sc1", 3, 1, 6, 0, 256)]
if os.environ.get("VARIANT_SET") == "map":
    # workgroup -> tile maps (sum2_map_kernel, mode 6; unroll = stripe KiB per operand, 0 = address
    # order): stripes dealt round-robin over the XCDs, against the shipped XCD-contiguous eighths
    VARIANTS = [("shipped", 3, 1, 1, 0, 256), ("map_address", 6, 0, 0, 0, 256)] + [
        ("stripe%dK" % kib, 6, kib, 0, 0, 256) for kib in
        [int(x) for x in os.environ.get("STRIPES_KIB", "256,1024,2048,4096,8192").split(",")]]
if os.environ.get("VARIANT_SET") == "focus":
    # round 6, under XCD stripes: the shapes / policies that led the wider sweeps, side by side
    # (the stripe size itself is TIPS_STRIPE_KIB, one value per process)
    VARIANTS = [("shipped", 3, 1, 1, 0, 256), ("t128", 3, 1, 1, 0, 128), ("t128_nt", 3, 1, 7, 0, 128), ("st_nt", 3, 1, 7, 0, 256),
                ("st_sc0nt", 3, 1, 13, 0, 256), ("cap8", 3, 1, 1, 20480, 256), ("t64_nt", 3, 1, 7, 0, 64),
                ("u2t128_nt", 3, 2, 7, 0, 128)]
for mib in SIZES:
    n = mib << 18
    sets = [(torch.randn(n, device="cuda"), torch.randn(n, device="cuda"), torch.empty(n, device="cuda"))
            for _ in range(4)]
    best = {}
    for rnd in range(ROUNDS):
        for name, mode, unroll, nt, blocks, threads in (VARIANTS if rnd % 2 == 0 else VARIANTS[::-1]):
            def launch(i):
                a, b, c = sets[i % 4]
                rc = D.tips_sum_variant(c.data_ptr(), a.data_ptr(), b.data_ptr(), n, _lib.FLOAT32, mode, unroll, nt,
                                        blocks, threads, s.cuda_stream)
                assert rc == 0, (name, rc)
            for i in range(8):
                launch(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            K = 40
            e0.record(s)
            for i in range(K):
                launch(i)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / K * 1e3
            best[name] = min(us, best.get(name, us))
    a, b, c = sets[0]
    ok = bool(torch.equal(c, a + b))  # (the last launch of the last variant wrote set 3; set 0 earlier)
    for name, *_ in VARIANTS:
        us = best[name]
        print(json.dumps({"operand_MiB": mib, "variant": name, "us_per_launch": round(us, 2),
                          "frac_of_8TBps": round(3 * n * 4 / us / 1e6 / 8.0, 4), "check": ok}), flush=True)
    del sets
    torch.cuda.empty_cache()
