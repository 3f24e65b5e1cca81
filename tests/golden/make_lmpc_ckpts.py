"""Convert the reference's two CartPole-LMPC trained EMA state dicts (d=1, C=4, N=25,
ConditionedTemporalUnet base 32 / dim_mults (1, 2, 4)) to safetensors fixtures, with their args.yaml, so the
GPU box (which has no /root/reference) can run them through the HIP path:
  trained_models/2406400_models/1000000                  -> lmpc_2406400_1000000_ema.safetensors
  trained_models/420000_models_with_noisy_data/230000     -> lmpc_420000_noisy_230000_ema.safetensors
The checkpoints are loaded weights-only (tensor data, no code execution)."""
import os
import shutil

import torch
from safetensors.torch import save_file

REF = "/root/reference/trained_models/"
HERE = os.path.dirname(os.path.abspath(__file__))
MODELS = {"lmpc_2406400_1000000": "2406400_models/1000000",
          "lmpc_420000_noisy_230000": "420000_models_with_noisy_data/230000"}

if __name__ == "__main__":
    for name, sub in MODELS.items():
        src = os.path.join(REF, sub, "checkpoints", "ema_model_current_state_dict.pth")
        sd = torch.load(src, map_location="cpu", weights_only=True)
        dst = os.path.join(HERE, f"{name}_ema.safetensors")
        save_file({k: v.contiguous().float() for k, v in sd.items()}, dst,
                  metadata={"source": f"trained_models/{sub}/checkpoints/ema_model_current_state_dict.pth "
                                      "(weights-only load, fp32)"})
        shutil.copyfile(os.path.join(REF, sub, "args.yaml"), os.path.join(HERE, f"{name}_args.yaml"))
        print(dst, os.path.getsize(dst))
