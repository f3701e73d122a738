"""Seeded synthetic photon maps / queries for k-NN parity tests."""
import numpy as np

from gi_amd import PHOTON_DTYPE, QUERY_DTYPE


def photon_map(n, seed=0, box=1.1):
    """Photons on the 6 faces of a box (like a Cornell box photon map) with random power."""
    rng = np.random.default_rng(seed)
    ph = np.zeros(n, dtype=PHOTON_DTYPE)
    face = rng.integers(0, 6, n)
    pts = rng.random((n, 3)) * box
    axis = face % 3
    pts[np.arange(n), axis] = np.where(face < 3, 0.0, box)
    ph["pos"] = pts.astype(np.float32)
    ph["rgbe"][:, :3] = rng.integers(1, 256, (n, 3))
    ph["rgbe"][:, 3] = rng.integers(100, 130, n)
    ph["dir"] = rng.integers(0, 65536, n)
    return ph


def queries(n, seed=1, box=1.1, k=50, r=2.5, filt=0, spec=False):
    rng = np.random.default_rng(seed)
    q = np.zeros(n, dtype=QUERY_DTYPE)
    face = rng.integers(0, 6, n)
    pts = rng.random((n, 3)) * box
    axis = face % 3
    pts[np.arange(n), axis] = np.where(face < 3, 0.0, box)
    q["point"] = pts
    nrm = np.zeros((n, 3))
    nrm[np.arange(n), axis] = np.where(face < 3, 1.0, -1.0)
    q["normal"] = nrm
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    q["exact_bounce"] = v
    q["cos_theta"] = rng.choice([-0.7, 0.4, 0.9], n)
    q["kd"] = rng.random((n, 3))
    q["ks"] = rng.random((n, 3)) if spec else 0.0
    q["shininess"] = 10.0
    q["max_dist"] = r
    q["k"] = k
    q["filter"] = filt
    return q
