#!/usr/bin/env python3
"""Grouped skinny-GEMM tile shapes on the vae_large per-step products:
64-wide N tiles on 4 waves (256 threads) vs 128-wide tiles on 8 waves (512
threads, csrc/skinny_gemm.hip skr_skinny_gemm_group bn=128), over split-K
factors. HIP-graph replays of 50 back-to-back launches (each time includes
one kernel boundary). One JSON line per (product, bn, splits)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd.ops import gemm  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402

B, H, Hh = 100, 2048, 256
K, G, Gh = H + Hh, 4 * H, 4 * Hh


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return best


def main():
    dev = "cuda"
    bf = torch.bfloat16
    r = lambda *s: (torch.randn(*s, device=dev) * 0.1).to(bf)   # noqa: E731
    A, WhT, WyT = r(B, K), r(G, H), r(Gh, K)
    dRM, Whl, dRY, Wyl, dVEC, Pl = r(B, G), r(H, G), r(B, Gh), r(K, Gh), r(B, 12 * H), r(Hh, 12 * H)
    cases = {
        "fwd R_main+R_hyp": lambda s: [(A[:, :H], WhT, s[0]), (A, WyT, s[1])],
        "bwd dR_main W_h^T": lambda s: [(dRM, Whl, s[0])],
        "bwd dvec P^T": lambda s: [(dVEC, Pl, s[0])],
        "bwd dR_hyp W_y^T": lambda s: [(dRY, Wyl, s[0])],
    }
    plans = {   # (bn, splits, ring depth)
        "fwd R_main+R_hyp": [(64, (2, 4), 3), (64, (2, 4), 4), (64, (2, 4), 6), (64, (1, 4), 6), (64, (1, 6), 6),
                             (64, (1, 9), 6), (64, (1, 4), 3), (64, (1, 6), 4)],
        "bwd dR_main W_h^T": [(64, (8,), 3), (64, (8,), 4), (64, (8,), 6), (64, (4,), 6)],
        "bwd dvec P^T": [(64, (32,), 3), (64, (64,), 3), (64, (64,), 6), (64, (32,), 6)],
        "bwd dR_hyp W_y^T": [(64, (4,), 3), (64, (4,), 6), (64, (8,), 6)],
    }
    for name, mk in cases.items():
        for bn, splits, ns in plans[name]:
            jobs = []
            for (a, bt, S) in mk(splits):
                jobs.append((a, bt, torch.empty(S, B, bt.shape[0], device=dev), S))
            gemm.GROUP_BN = bn
            from sketch_rnn_amd.utils import native
            assert native.require_hip().lib.skr_gemm_set_nstage(ns) == 0
            try:
                us = timeit(lambda: gemm.rec_gemm_group(jobs))
                ok = all(((o.sum(0) - a.float() @ bt.float().t()).abs().max().item()
                          <= 1e-2 * (a.float() @ bt.float().t()).abs().max().item() + 1e-3) for a, bt, o, _ in jobs)
            except RuntimeError as e:
                us, ok = -1.0, str(e)
            wg = sum((bt.shape[0] // bn) * S for _, bt, _, S in jobs)
            print(json.dumps({"product": name, "bn": bn, "ns": ns, "splits": list(splits), "workgroups": wg,
                              "us": round(us, 2), "correct": ok}), flush=True)
    gemm.GROUP_BN = 0
    native.require_hip().lib.skr_gemm_set_nstage(3)


if __name__ == "__main__":
    main()
