"""Drop-in for the reference's envs/physics.py (collide_sphere_with_moving_plane, :3-23).

The collision runs on the device through libpongmi (pm_collide, the same fp64 device function
every env tick uses). `collide_batch` evaluates many rows in one launch; the scalar entry point
keeps the reference signature (one launch per call, the result read from host-mapped memory)."""
import ctypes

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


_slot = None
_call = None  # (pm_collide1, launch stream handle, the stream object kept alive), made on the first call


def collide_sphere_with_moving_plane(vn, vt, u, omega, e, mu, m, R):
    """One launch (pm_collide1: the row as kernel arguments, the result written into a host-mapped
    buffer the host polls), no copies, no stream synchronisation."""
    global _slot, _call
    if _slot is None:
        _slot = _lib.MappedSlot(8, 6)  # vn' vt' omega' (fp64) | seq
        st = _lib.current_stream()
        _call = (_lib.load().pm_collide1, st.cuda_stream, st)
    row = (ctypes.c_double * 8)(vn, vt, u, omega, e, mu, m, R)
    inertia = (2 / 5) * m * R ** 2  # CPython's I (:9)
    rc = _call[0](row, inertia, _slot.dev, _slot.next_seq(), _call[1])
    if rc:
        _lib.check(rc, "pm_collide1")
    _slot.wait()
    vn2, vt2, om2 = _slot.f64[0:3].tolist()
    return vn2, vt2, om2
