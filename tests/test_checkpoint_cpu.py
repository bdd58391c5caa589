"""Checkpoint compatibility with the reference (runners/InterTrainer.py:867-960).

tests/golden/ckpt_manifest.json (G10, make_golden.py) is the manifest of the file the
reference's save_checkpoint wrote after the G4 training step: top-level keys, every
coarse_model state_dict entry in order (dtype, shape, sum, sum of squares) and the
torch.optim.Adamax state_dict (param_groups, per-index state).  The ~120 MB file itself is
rebuilt here from the oracle's step (pinned to the reference by G4), checked entry by entry
against the manifest, written with torch.save, and loaded through InterTrainer's
load_checkpoint exactly as a reference checkpoint would be (weights_only=True)."""
import json
import os
import types

import numpy as np
import pytest
import torch

import inputs
from oracle import hrnet as O
from oracle import losses as OL
from oracle import step as OS

G = os.path.join(os.path.dirname(__file__), "golden")


def manifest():
    with open(os.path.join(G, "ckpt_manifest.json")) as f:
        return json.load(f)


def _close(t, st):
    assert str(t.dtype).replace("torch.", "") == st["dtype"] and list(t.shape) == st["shape"]
    s, q = float(t.double().sum()), float((t.double() ** 2).sum())
    return abs(s - st["sum"]) <= 1e-5 * max(1.0, abs(st["sum"])) and abs(q - st["sumsq"]) <= 1e-5 * max(1.0, st["sumsq"])


def reference_checkpoint(step_as_int=False):
    """(dict laid out as the reference's save_dict, oracle (params, adamax state)) after the
    G4 step.  step_as_int: torch 1.0.1's Adamax stored 'step' as a Python int."""
    man = manifest()
    P = O.init_params(1024)
    data = inputs.step_batch(2, 32, 64)
    _, _, new, state, _ = OS.inter_step(P, OL.synthetic_vgg19_state(), data)
    names = [k for k, _ in man["coarse_model"]]
    sd = {k: new[k].detach().clone() for k in names}
    groups = [dict(g) for g in man["coarse_opt"]["param_groups"]]
    for g in groups:
        g["betas"] = tuple(g["betas"])
    st = {}
    for i, k in enumerate(names):
        s = state[k]
        st[i] = {"step": (int(s["step"]) if step_as_int else torch.tensor(float(s["step"]))),
                 "exp_avg": s["exp_avg"].detach().clone(), "exp_inf": s["exp_inf"].detach().clone()}
    ck = {"session": man["session"], "epoch": man["epoch"], "coarse_model": sd,
          "coarse_opt": {"state": st, "param_groups": groups}}
    return ck, (new, state)


def test_rebuilt_checkpoint_matches_reference_manifest():
    man = manifest()
    ck, _ = reference_checkpoint()
    assert list(ck.keys()) == man["top_keys"]
    assert [k for k in ck["coarse_model"]] == [k for k, _ in man["coarse_model"]]
    bad = [k for k, st in man["coarse_model"] if not _close(ck["coarse_model"][k], st)]
    assert not bad, bad[:5]
    for i, sts in man["coarse_opt"]["state"].items():
        for k, st in sts.items():
            v = ck["coarse_opt"]["state"][int(i)][k]
            assert _close(v, st), (i, k)
    assert len(ck["coarse_opt"]["param_groups"][0]["params"]) == len(man["coarse_model"])


def _trainer_loading(tmp_path, ck, split="train"):
    from deep_video_interpolation_extrapolation_amd.options import default_args
    from deep_video_interpolation_extrapolation_amd.runners.InterTrainer import InterTrainer
    man = manifest()
    os.makedirs(tmp_path / "checkpoint", exist_ok=True)
    torch.save(ck, tmp_path / "checkpoint" / man["file"])
    args = default_args("INTER", syn_type="inter", train_coarse=True, load_coarse=True, resume=split == "train",
                        checksession=1, checkepoch=1, checkpoint=0, load_dir=str(tmp_path), batch_size=2,
                        input_h=32, input_w=64, precision="fp32", synthetic=2, num_workers=0, split=split)
    args.logger = types.SimpleNamespace(info=lambda *a: None)
    torch.manual_seed(0)  # a different init: every value must come from the file
    return InterTrainer(args)


@pytest.mark.parametrize("step_as_int", [False, True])
def test_inter_trainer_loads_reference_checkpoint(tmp_path, step_as_int):
    """weights, Adamax state and epoch bookkeeping of a reference checkpoint (torch 2.x and
    torch 1.0.1 'step' formats) land in the HIP trainer's flat buffers."""
    ck, (new, state) = reference_checkpoint(step_as_int)
    tr = _trainer_loading(tmp_path, ck)
    assert tr.epoch == 2  # resume: the file's epoch (l.954-956)
    named = dict(tr.model.module.coarse_model.named_parameters())
    for k, v in new.items():
        assert torch.equal(named[k].detach().cpu(), v.detach()), k
    opt_state = tr.coarse_opt.state
    for k, v in new.items():
        s = opt_state[named[k]]
        assert float(s["step"]) == 1.0
        assert torch.equal(s["exp_avg"].cpu(), state[k]["exp_avg"]) and torch.equal(s["exp_inf"].cpu(), state[k]["exp_inf"])


def test_val_split_loads_reference_checkpoint(tmp_path):
    """--split val: the reference loads the checkpoint without --r (l.105) and sets the
    epoch to the file's epoch - 1 (l.957-959)."""
    ck, (new, _) = reference_checkpoint()
    tr = _trainer_loading(tmp_path, ck, split="val")
    assert tr.epoch == 1
    named = dict(tr.model.module.coarse_model.named_parameters())
    k = next(iter(new))
    assert torch.equal(named[k].detach().cpu(), new[k].detach())
