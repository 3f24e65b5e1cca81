"""Convert the reference's trained Panda EMA state dict (trained_models/panda_test6_117600/final, SURVEY §8f
row 1: d=7 joint torques, C=20 context, H=128, N=25 exponential) to a safetensors fixture so the GPU box
(which has no /root/reference) can run the trained Panda net through the HIP path. Weights-only load
(tensor data, no code execution); the full-module pickles next to it are never opened."""
import os

import torch
from safetensors.torch import save_file

SRC = ("/root/reference/trained_models/panda_test6_117600/final/checkpoints/"
       "ema_model_current_state_dict.pth")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "panda_test6_117600_ema.safetensors")

if __name__ == "__main__":
    sd = torch.load(SRC, map_location="cpu", weights_only=True)
    save_file({k: v.contiguous().float() for k, v in sd.items()}, DST,
              metadata={"source": "trained_models/panda_test6_117600/final/checkpoints/"
                                  "ema_model_current_state_dict.pth (weights-only load, fp32)"})
    print(DST, os.path.getsize(DST))
