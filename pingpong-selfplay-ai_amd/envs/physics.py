"""Drop-in for the reference's envs/physics.py (collide_sphere_with_moving_plane, :3-23).

The collision runs on the device through libpongmi (pm_collide, the same fp64 device function
every env tick uses). `collide_batch` evaluates many rows in one launch; the scalar entry point
keeps the reference signature (one launch + one host round trip per call)."""
import numpy as np
import torch

from pongmi import _lib


def collide_batch(rows, device="cuda"):
    """rows [n, 8] = (vn, vt, u, omega, e, mu, m, R) -> [n, 3] = (vn', vt', omega') fp64."""
    rows = np.ascontiguousarray(rows, np.float64).reshape(-1, 8)
    inertia = np.array([(2 / 5) * m * R ** 2 for m, R in rows[:, 6:8]], np.float64)  # CPython's I (:9)
    d_in = torch.from_numpy(rows).to(device)
    d_I = torch.from_numpy(inertia).to(device)
    out = torch.empty((rows.shape[0], 3), dtype=torch.float64, device=device)
    _lib.check(_lib.load().pm_collide(d_in.data_ptr(), d_I.data_ptr(), out.data_ptr(), rows.shape[0],
                                      _lib.stream_ptr()), "pm_collide")
    return out.cpu().numpy()


def collide_sphere_with_moving_plane(vn, vt, u, omega, e, mu, m, R):
    vn2, vt2, om2 = collide_batch([[vn, vt, u, omega, e, mu, m, R]])[0]
    return float(vn2), float(vt2), float(om2)
