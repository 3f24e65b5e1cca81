"""CPU oracle for the diffusion-MPC hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-source restatement of the reference algorithm
(XuehuaOvO/MPC_via_Diffusion_Model, read as text; importing or running the
reference is denied for this build, see DESIGN.md "Oracle"). It exists so that
tests, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``
have something to check the HIP path against. The product package
(``mpc_via_diffusion_model_amd``) never imports it and fails loudly when its
HIP library is missing.

Pinning: the restatement reproduces the reference's
known-answer tests — KAT1 schedule values, KAT2 parameter counts, KAT3 the
trained ``cart_pole_84000_test1`` output trace, KAT5 the ``calMPCCost`` golden,
KAT6 the ZOH matrices — see ``tests/test_oracle_kats.py``.

Modules
  schedule   beta schedules + the 12 diffusion buffers (helpers.py, diffusion_model_base.py)
  layers     U-Net / MLP building blocks (mpd/models/layers/layers.py)
  nets       ConditionedTemporalUnet, TemporalUnet, the CFG MLP noise-net (temporal_unet.py)
  sampler    CFG-DDPM loop, DDIM, build-defined CFG-DDIM (diffusion_model_base.py, sample_functions.py)
  normalizer LimitsNormalizer semantics (mpd/datasets/normalization.py)
  systems    rollout dynamics + MPC costs in fp64 (scripts/inference, scripts/mpc_data_collecting)
  c/         the same rollout/cost in plain C (fp64), built by ``oracle/Makefile``
"""
