"""Check that the timing-only op-kind skip (DVIE_SKIP_KINDS, -DDVIE_TIMING_DBG library) takes
effect: one InterTrainer step at a small shape, printing the loss and a few gradient norms."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ.setdefault("DVIE_PRECISION", "bf16")
from bench import make_batch  # noqa: E402
from deep_video_interpolation_extrapolation_amd.options import default_args  # noqa: E402
from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer  # noqa: E402

dev = torch.device("cuda:0")
args = default_args("INTER", syn_type="inter", interval=5, mode="xs2xs", vid_length=1, train_coarse=True, batch_size=2,
                    input_h=64, input_w=128, precision="bf16", synthetic=2, num_workers=0, split="train", rank=0, gpus=1)
torch.manual_seed(1)
tr = InterTrainer(args)
data = make_batch(2, 64, 128, dev, 0)
ld = tr.forward_backward(data)
torch.cuda.synchronize()
m = tr.model.module.coarse_model
norms = {k: float(p.grad.norm()) for k, p in list(m.named_parameters())[:4] if p.grad is not None}
print("skip", os.environ.get("DVIE_SKIP_KINDS"), "loss", float(ld["loss_all"]), norms)
