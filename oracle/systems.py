"""ctypes front-end of the fp64 C rollout/cost oracle (oracle/c/mpc_oracle.c) — test infrastructure only.

``build()`` compiles it with ``make -C oracle``; tests, ``smoke()`` and bench's cpu_baseline load it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmpcoracle.so")
_lib = None

SYSTEMS = {"cartpole_lin5": 0, "cartpole_nl5": 1, "cartpole_zoh4": 2, "double_int2d": 3, "pendulum": 4,
           "quadrotor12": 5}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        L.oracle_rollout_cost.argtypes = [ctypes.c_int, dp, dp, ctypes.c_int64, ctypes.c_int, dp]
        L.oracle_rollout_cost.restype = ctypes.c_int
        L.oracle_argmin.argtypes = [dp, ctypes.c_int64]
        L.oracle_argmin.restype = ctypes.c_int64
        L.oracle_step.argtypes = [ctypes.c_int, dp, dp, dp]
        L.oracle_step.restype = ctypes.c_int
        L.oracle_system_info.argtypes = [ctypes.c_int, ip, ip, ip, dp, dp, dp, dp]
        L.oracle_system_info.restype = ctypes.c_int
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def system_info(name):
    nx, nu, ck = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    Q, R, P, xr = (np.zeros(n) for n in (12, 4, 12, 12))
    if lib().oracle_system_info(SYSTEMS[name], nx, nu, ck, _dp(Q), _dp(R), _dp(P), _dp(xr)):
        raise ValueError(name)
    return dict(nx=nx.value, nu=nu.value, cost_kind=ck.value, Q=Q[:nx.value], R=R[:nu.value], P=P[:nx.value],
                xref=xr[:nx.value])


def step(name, x, u):
    x = np.ascontiguousarray(x, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    xn = np.zeros(12)
    lib().oracle_step(SYSTEMS[name], _dp(x), _dp(u), _dp(xn))
    return xn[:x.shape[0]]


def rollout_cost(name, x0, u):
    """x0: [nx] fp64; u: [B, H, nu] (already unnormalised; cast exactly to fp64). Returns cost [B] fp64."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    B, H = u.shape[0], u.shape[1]
    cost = np.zeros(B)
    if lib().oracle_rollout_cost(SYSTEMS[name], _dp(x0), _dp(u), B, H, _dp(cost)):
        raise ValueError("oracle_rollout_cost failed")
    return cost


def argmin(cost):
    c = np.ascontiguousarray(cost, dtype=np.float64)
    return int(lib().oracle_argmin(_dp(c), c.shape[0]))
