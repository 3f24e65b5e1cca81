"""System table for the rollout/cost kernel.

Each constant is computed with the same Python fp64 expression (same association, left to right)
the reference evaluates at run time, so the kernel's arithmetic rounds exactly like the reference's
numpy code. ``params`` layouts match the ``dyn_step`` switch in csrc/rollout.hip.
"""
import math
from dataclasses import dataclass, field

import numpy as np

from . import _native as N

CARTPOLE_LIN5, CARTPOLE_NL5, CARTPOLE_ZOH4, DOUBLE_INT2D, PENDULUM, QUADROTOR12 = range(6)


@dataclass
class System:
    name: str
    system: int
    cost_kind: int
    n_x: int
    n_u: int
    params: list
    Q: list
    R: list
    P: list
    x_ref: list = field(default_factory=list)
    reference: str = ""

    def desc(self):
        d = N.SystemDesc()
        d.system, d.cost_kind, d.n_x, d.n_u = self.system, self.cost_kind, self.n_x, self.n_u
        for i, v in enumerate(self.params):
            d.params[i] = v
        for i in range(self.n_x):
            d.Q[i] = self.Q[i]
            d.P[i] = self.P[i]
            d.x_ref[i] = self.x_ref[i] if self.x_ref else 0.0
        for i in range(self.n_u):
            d.R[i] = self.R[i]
        return d


def cartpole_lin5():
    """EulerForwardCartpole_virtual with the linearised xdot_new + calMPCCost
    (scripts/inference/Cart_Diffusion_inference.py:37-46 weights, :122-130 constants, :168-197, :247-283)."""
    M_car, m_pole, l_pendul, k, c, G = 4.5, 0.12, 0.14, 0.5, 0.002, 9.81
    I = (m_pole * l_pendul ** 2) / 3
    v_1 = (M_car + m_pole) / (I * (M_car + m_pole) + (l_pendul ** 2) * m_pole * M_car)
    v_2 = (I + (l_pendul ** 2) * m_pole) / (I * (M_car + m_pole) + (l_pendul ** 2) * m_pole * M_car)
    TS = 0.01
    params = [
        TS,
        -k * v_2,
        ((l_pendul * m_pole) ** 2) * G * v_2 / (I + (l_pendul ** 2) * m_pole),
        l_pendul * m_pole * c * v_2 / (I + (l_pendul ** 2) * m_pole),
        v_2,
        -l_pendul * m_pole * k * v_1 / (M_car + m_pole),
        l_pendul * m_pole * G * v_1,
        c * v_1,
        l_pendul * m_pole * v_1 / (M_car + m_pole),
        2 / np.pi,
        np.pi,
    ]
    q = [0.01, 0.01, 0.0, 0.001, 1000.0]
    return System("cartpole_lin5", CARTPOLE_LIN5, N.MPCD_COST_CALMPC, 5, 1, params, q, [0.1], list(q),
                  reference="scripts/inference/Cart_Diffusion_inference.py:168-197,247-283")


def cartpole_nl5():
    """Nonlinear Euler cart-pole + the NMPC data-collection objective
    (scripts/mpc_data_collecting/nmpc_multi_process_collect_data.py:63-65, :96-111, :121-137, :143-172)."""
    M_CART, M_POLE, L_POLE, G = 2.0, 1.0, 1.0, 9.81
    M_TOTAL = M_CART + M_POLE
    MPLP, MPG, MTG, MTLP = M_POLE * L_POLE, M_POLE * G, M_TOTAL * G, M_TOTAL * G
    params = [0.01, MPLP, MPG, M_TOTAL, M_POLE, MTG, MTLP, 2 / np.pi, np.pi]
    return System("cartpole_nl5", CARTPOLE_NL5, N.MPCD_COST_CANONICAL, 5, 1, params,
                  [0.01, 0.01, 0.0, 0.01, 1000.0], [0.001], [0.01, 0.1, 0.0, 0.1, 1000.0],
                  reference="scripts/mpc_data_collecting/nmpc_multi_process_collect_data.py:121-172")


# c2d(A, B, Ts=0.1, 'zoh') of Diffusion_MPC_Inference.py:39-84 = expm([[A, B], [0, 0]] * Ts) (SURVEY KAT6)
ZOH_A = [[1.0, 0.09949537483382852, 0.015327761653922887, 0.0005062874425049262],
         [0.0, 0.9897973187953647, 0.3136747477766333, 0.015327761653922889],
         [0.0, -0.0025546269423204816, 1.1535307602604814, 0.10506917464734186],
         [0.0, -0.05227912462943889, 3.144411358593294, 1.1535307602604812]]
ZOH_B = [0.010029501100503806, 0.20152218688018167, 0.025461888182787322, 0.5202366193520683]


def cartpole_zoh4():
    """Linear ZOH cart-pole, cost Q=diag(10,1,10,1), R=1, P=diag(100,1,100,1)
    (scripts/inference/Diffusion_MPC_Inference.py:39-84, :313-315, :357-371)."""
    params = [v for row in ZOH_A for v in row] + list(ZOH_B)
    return System("cartpole_zoh4", CARTPOLE_ZOH4, N.MPCD_COST_CANONICAL, 4, 1, params, [10.0, 1.0, 10.0, 1.0],
                  [1.0], [100.0, 1.0, 100.0, 1.0], reference="scripts/inference/Diffusion_MPC_Inference.py:39-84")


def double_int2d(dt=0.1):
    """BUILD-DEFINED (no reference): planar double integrator x=[px,py,vx,vy], u=[ax,ay]."""
    return System("double_int2d", DOUBLE_INT2D, N.MPCD_COST_CANONICAL, 4, 2, [dt, 0.5 * dt * dt],
                  [1.0, 1.0, 0.1, 0.1], [0.01, 0.01], [10.0, 10.0, 1.0, 1.0], reference="build-defined")


def pendulum(dt=0.05):
    """BUILD-DEFINED (no reference): damped pendulum swing-up to theta = pi."""
    return System("pendulum", PENDULUM, N.MPCD_COST_CANONICAL, 2, 1, [dt, 9.81 / 1.0, 0.1, 1.0 / (1.0 * 1.0 * 1.0)],
                  [10.0, 0.1], [0.01], [100.0, 1.0], x_ref=[math.pi, 0.0], reference="build-defined")


def quadrotor12(dt=0.02):
    """BUILD-DEFINED (no reference): 12-state rigid-body quadrotor, hover at the origin."""
    q = [10, 10, 10, 1, 1, 1, 1, 1, 1, 0.1, 0.1, 0.1]
    return System("quadrotor12", QUADROTOR12, N.MPCD_COST_CANONICAL, 12, 4, [dt, 1.0, 9.81, 0.01, 0.01, 0.02],
                  [float(v) for v in q], [0.1, 1.0, 1.0, 1.0], [10.0 * v for v in q], reference="build-defined")


REGISTRY = {f.__name__: f for f in (cartpole_lin5, cartpole_nl5, cartpole_zoh4, double_int2d, pendulum, quadrotor12)}


def get(name):
    return REGISTRY[name]()
