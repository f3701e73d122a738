#!/usr/bin/env python3
"""Offline analysis of a caustic_fb_dump.py file (CPU, scipy): why queries reach the caustic
k-NN's query-per-wave fallback. Per sampled fallback query: d_K (K-th neighbour distance, inf
when fewer than K photons lie within r), the leaf start bound U = min over q's kd leaf of
|q - p| + d_K(p), and the photon counts within d_K, U and r.

usage: tools/caustic_fb_analyze.py gpurun_out/fb/c2.npz [--K 225 --r 0.225 --n 100000]
"""
import argparse

import numpy as np
from scipy.spatial import cKDTree


def leaf_of(q, nodes, L):
    node = np.ones(len(q), dtype=np.int64)
    ax_bits = nodes[:, 7].view(np.int32)
    while True:
        m = node < L
        if not m.any():
            break
        nd = node[m]
        ax = ax_bits[nd]
        qa = q[m, :][np.arange(m.sum()), ax]
        node[m] = 2 * nd + ((qa - nodes[nd, 3]) >= 0)
    return node - L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--K", type=int, default=225)
    ap.add_argument("--r", type=float, default=0.225)
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--which", default="fb")
    a = ap.parse_args()
    z = np.load(a.npz)
    P = z["photons"].astype(np.float64)
    nodes, L = z["nodes"], int(z["nleaves"])
    N = len(P)
    hdr = z["hdr"]
    print(f"launch nq {hdr[0]} second-pass {hdr[1]} fallback {hdr[2]}; photons {N}, leaves {L} "
          f"({N / L:.0f} per leaf)")
    Q = z[a.which].astype(np.float64)
    rng = np.random.default_rng(1)
    sel = np.sort(rng.choice(len(Q), size=min(a.n, len(Q)), replace=False))
    Q = Q[sel]
    T = cKDTree(P)
    K, r = a.K, a.r
    # per-photon d_K (only the photons in the queries' leaves are needed)
    lf = leaf_of(Q, nodes, L)
    s0 = (lf * N) // L
    s1 = ((lf + 1) * N) // L
    need = np.unique(np.concatenate([np.arange(x, y) for x, y in zip(*np.unique(np.stack([s0, s1], 1), axis=0).T)]))
    dkp = np.full(N, np.inf)
    d, _ = T.query(P[need], k=K, distance_upper_bound=r, workers=8)
    dkp[need] = d[:, K - 1]
    dq, _ = T.query(Q, k=K, distance_upper_bound=r, workers=8)
    dK = dq[:, K - 1]
    nr = T.query_ball_point(Q, r, workers=8, return_length=True)
    U = np.empty(len(Q))
    for i in range(len(Q)):
        pp = P[s0[i]:s1[i]]
        U[i] = np.min(np.sqrt(((pp - Q[i]) ** 2).sum(1)) + dkp[s0[i]:s1[i]])
    U = np.minimum(U, r)
    nU = T.query_ball_point(Q, U, workers=8, return_length=True)
    sparse = ~np.isfinite(dK)
    print(f"sampled {len(Q)} of {a.which}: sparse (< K within r) {sparse.mean():.3f}")
    print(f"  photons within r: median {np.median(nr):.0f}, p10 {np.percentile(nr, 10):.0f}, "
          f"p90 {np.percentile(nr, 90):.0f}")
    dense = ~sparse
    if dense.any():
        ratio = (U[dense] / dK[dense]) ** 2
        print(f"  dense: (U/d_K)^2 median {np.median(ratio):.2f} p90 {np.percentile(ratio, 90):.2f}; "
              f"photons within U median {np.median(nU[dense]):.0f} p90 {np.percentile(nU[dense], 90):.0f}"
              f"; d_K median {np.median(dK[dense]):.4g}")
        qd, _ = T.query(Q[dense], k=1)
        print(f"  nearest photon / d_K: median {np.median(qd / dK[dense]):.3f}")
    if sparse.any():
        print(f"  sparse: photons within r median {np.median(nr[sparse]):.0f}, "
              f"U = r fraction {(U[sparse] >= r).mean():.3f}")
    for lo, hi in [(0, 256), (256, 512), (512, 1024), (1024, 4096), (4096, 1 << 30)]:
        m = (nU >= lo) & (nU < hi)
        print(f"  photons within U in [{lo}, {hi}): {m.mean():.3f}")


if __name__ == "__main__":
    main()
