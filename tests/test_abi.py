"""C ABI: libmpcd.so loads, exports every entry point include/mpcd.h declares, and its host-side
logic (parameter spec, argument checks, error reporting) behaves. No GPU needed."""
import ctypes
import os
import re

import pytest
import torch

from mpc_via_diffusion_model_amd import NetSpec
from mpc_via_diffusion_model_amd import _native as N
from oracle import nets

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "mpcd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mpcd_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = N.lib()
    fns = header_functions()
    assert len(fns) >= 14
    for f in fns:
        assert hasattr(lib, f), f"libmpcd.so does not export {f}"
    assert set(fns) <= set(N.EXPORTS), "ctypes binding is missing a header function"


def test_library_is_gfx950_code_object():
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("spec,module", [
    (NetSpec("mlp", 2, 32, 4), lambda: nets.ConditionedMLPNet(state_dim=2, horizon=32, context_dim=4)),
    (NetSpec("mlp", 2, 16, 4), lambda: nets.ConditionedMLPNet(state_dim=2, horizon=16, context_dim=4)),
    (NetSpec("unet", 1, 32, 5), lambda: nets.ConditionedTemporalUnet(state_dim=1, context_dim=5)),
    (NetSpec("unet", 7, 128, 20), lambda: nets.ConditionedTemporalUnet(state_dim=7, context_dim=20)),
    (NetSpec("unet", 1, 32, 0, cfg=False), lambda: nets.TemporalUnet(state_dim=1, dim_mults=(1, 2, 4))),
    (NetSpec("unet", 2, 64, 3, cfg=False, dim_mults=(1, 2, 4, 8)),
     lambda: nets.TemporalUnet(state_dim=2, dim_mults=(1, 2, 4, 8), conditioning_type="default",
                               conditioning_embed_dim=3)),
])
def test_param_spec_is_state_dict_order(spec, module):
    sd = module().state_dict()
    ps = N.param_spec(spec.desc())
    assert [n for n, _ in ps] == list(sd.keys())
    assert all(tuple(sd[n].shape) == s for n, s in ps)


def test_param_count_and_errors():
    d = NetSpec("unet", 1, 32, 5).desc()
    nt, nf = ctypes.c_int32(), ctypes.c_int64()
    assert N.lib().mpcd_net_param_count(ctypes.byref(d), ctypes.byref(nt), ctypes.byref(nf)) == 0
    assert nf.value == 1000929
    bad = NetSpec("unet", 1, 32, 5).desc()
    bad.kind = 7
    assert N.lib().mpcd_net_param_count(ctypes.byref(bad), ctypes.byref(nt), ctypes.byref(nf)) == -1
    assert b"kind" in N.lib().mpcd_last_error()
    with pytest.raises(N.MpcdError):
        N.check(-5, "probe")


def test_create_without_gpu_reports_error():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = ctypes.c_void_p()
    rc = N.lib().mpcd_create(0, ctypes.byref(ctx))
    assert rc != 0 and N.lib().mpcd_last_error()


def test_gemm_numerics_selection_is_validated():
    """dtype: f32 and f32x3 accepted for both nets, f16 for the U-Net only (MLP f16 is MPCD_EUNSUP, -5);
    unknown names are rejected on the host."""
    nt, nf = ctypes.c_int32(), ctypes.c_int64()
    L = N.lib()
    assert N.MPCD_F32X3 == 2
    for spec, want in ((NetSpec("mlp", 2, 32, 4, dtype="f32x3"), 0), (NetSpec("mlp", 2, 32, 4), 0),
                       (NetSpec("unet", 1, 32, 5, dtype="f32x3"), 0), (NetSpec("unet", 4, 64, 12, dtype="f16"), 0),
                       (NetSpec("mlp", 2, 32, 4, dtype="f16"), -5)):
        d = spec.desc()
        assert L.mpcd_net_param_count(ctypes.byref(d), ctypes.byref(nt), ctypes.byref(nf)) == want, spec
    with pytest.raises(ValueError):
        NetSpec("mlp", 2, 32, 4, dtype="bf16").desc()


def test_trainer_argument_checks():
    """mpcd_trainer_create rejects bad arguments on the host, before any device work."""
    L = N.lib()
    cfg = N.TrainCfg(3e-3, 0.9, 0.999, 1e-8, 0.995, 1000, 10)
    sched = (ctypes.c_float * 10)(*([0.5] * 10))
    tr = ctypes.c_void_p()
    d = NetSpec("mlp", 2, 16, 4).desc()
    nt, nf = ctypes.c_int32(), ctypes.c_int64()
    assert L.mpcd_net_param_count(ctypes.byref(d), ctypes.byref(nt), ctypes.byref(nf)) == 0
    params = (ctypes.c_float * (nf.value + 1))()
    # wrong parameter count
    assert L.mpcd_trainer_create(ctypes.byref(d), params, nf.value + 1, ctypes.byref(cfg), sched, sched, 10,
                                 ctypes.byref(tr)) == -1
    assert b"floats" in L.mpcd_last_error()
    # no schedule
    assert L.mpcd_trainer_create(ctypes.byref(d), params, nf.value, ctypes.byref(cfg), None, sched, 10,
                                 ctypes.byref(tr)) == -1
    # the 3-arg TemporalUnet has no CFG mask to train with
    u = NetSpec("unet", 1, 32, 0, cfg=False).desc()
    assert L.mpcd_trainer_create(ctypes.byref(u), params, nf.value, ctypes.byref(cfg), sched, sched, 10,
                                 ctypes.byref(tr)) == -5
    assert not tr.value
    assert L.mpcd_trainer_step(None, None, None, None, None, None, 0, 1, None, None) == -1
