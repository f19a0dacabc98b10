"""``import osqp`` shim: routes the reference's ``osqp.OSQP()`` to the MI355X solver.

Put this directory first on ``sys.path`` (or PYTHONPATH) together with
``python-mpc_amd`` and the reference's own scripts run unmodified:
``prob = osqp.OSQP(); prob.setup(P, q, A, l, u, warm_start=True)``,
``prob.update(q=..., l=..., u=...)``, ``res = prob.solve()`` and ``res.x``,
``res.y``, ``res.info.status``, ``res.info.iter`` behave as in osqp-python 0.6
(vehicle_lateral_mpc_slack_increment.py:118-121,237,248,252,256,269;
Control/MPC/mpc_kinematics.py:194-198; Control/MPC/mpc_dynamics.py:240-244,392-396).
"""
from osqp_amd import OSQP, constant  # noqa: F401

__version__ = "0.6.2+mpcqp"
