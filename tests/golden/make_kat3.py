"""Convert the reference's trained EMA state dict (cart_pole_84000_test1) to a
safetensors fixture so the GPU box (which has no /root/reference) can run KAT3 through the HIP path.
The checkpoint is loaded weights-only (tensor data, no code execution); the full-module pickles next
to it are never opened."""
import os

import torch
from safetensors.torch import save_file

SRC = ("/root/reference/trained_models/cart_pole_84000_test1/final/checkpoints/"
       "ema_model_current_state_dict.pth")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cart_pole_84000_test1_ema.safetensors")

if __name__ == "__main__":
    sd = torch.load(SRC, map_location="cpu", weights_only=True)
    save_file({k: v.contiguous().float() for k, v in sd.items()}, DST,
              metadata={"source": "trained_models/cart_pole_84000_test1/final/checkpoints/"
                                  "ema_model_current_state_dict.pth (weights-only load, fp32)"})
    print(DST, os.path.getsize(DST))
