"""A CPU stand-in for osqp_amd.DeviceBatch -- TEST INFRASTRUCTURE ONLY.

tests/test_multiproc.py runs bench.main() on CPU ranks (gloo) to rehearse the
multi-GPU rank logic (launcher, shards, barrier + max-over-ranks timing, the JSON
line) without a GPU.  This class has DeviceBatch's methods and answers them with the
CPU oracle on torch CPU tensors.  The product never imports it; bench.py only uses it
when a test passes it in (bench.main(solver_cls=...)).
"""
import numpy as np

import pyoracle


class FakeBatch:
    def __init__(self, P, A, B, device=0, **settings):
        self.P, self.A, self.B = P, A, int(B)
        self.settings = settings
        self.n, self.m = P.shape[0], A.shape[0]
        self._timing = False
        self._n_solve = 0
        self._data = None

    def setup(self, Px, Ax, q, l, u, stream=None):
        self._data = [t.numpy() for t in (Px, Ax, q, l, u)]

    def solve(self, x=None, y=None, status=None, iters=None, stream=None):
        Px, Ax, q, l, u = self._data
        r = pyoracle.solve_batch(self.P, self.A, Px, q, Ax, l, u, nthreads=1, **self.settings)
        for t, v in ((x, r.x), (y, r.y), (status, r.status_val), (iters, r.iter)):
            if t is not None:
                t.copy_(__import__("torch").from_numpy(np.ascontiguousarray(v)))
        self._n_solve += int(self._timing)

    def setup_solve(self, Px, Ax, q, l, u, x=None, y=None, status=None, iters=None, stream=None):
        self.setup(Px, Ax, q, l, u)
        self.solve(x, y, status, iters)

    def warm_start(self, x=None, y=None, stream=None):
        raise NotImplementedError("the CPU stand-in rehearses cold solves only")

    def synchronize(self):
        pass

    def timing(self, enable=True, setup=True):
        self._timing = bool(enable)
        if enable:
            self._n_solve = 0

    def timing_read(self):
        return dict(setup_ms=0.0, n_setup=0, solve_ms=1.0 * self._n_solve, n_solve=self._n_solve)

    def plan_info(self):
        return dict(nb=4, block=32, amax=5, npad=128, lds_bytes_solve=0, variant=-1, threads_per_qp=0)
