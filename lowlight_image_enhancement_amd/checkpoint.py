"""Checkpoint compatibility with the reference's training harness.

Reference: NAFNet_base/basicsr/models/base_model.py
  * save_network (:195-225): ``torch.save({param_key: state_dict (on CPU, 'module.' stripped)}, f'{label}_{iter}.pth')``
  * load_network (:262-287): ``torch.load`` -> ``[param_key]`` -> strip 'module.' -> ``load_state_dict(strict)``
  * save_training_state (:290-314): ``{'epoch', 'iter', 'optimizers': [opt.state_dict()], 'schedulers': [...]}``
    written as ``f'{iter}.state'``
  * resume_training (:316-333): optimizer / scheduler ``load_state_dict``

The network side is exact: ``NAFNet.state_dict()`` already presents the reference keys, shapes and layouts, so a
``net_g_*.pth`` file written here loads into the reference NAFNet and vice versa.  The optimizer side is written in
``torch.optim.AdamW.state_dict()`` form over the reference parameter order (``net.ref_order`` = registration order),
so the reference's AdamW resumes from it; the flat fused-AdamW state (``NBPTrainer.exp_avg`` / ``exp_avg_sq``) is
converted to and from that per-parameter form.  Files are read with ``weights_only=True`` (no unpickling of code).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, Optional

import torch

from .nafnet import NAFNet


def _bare(net):
    return net.module if hasattr(net, "module") else net


def save_network(net, path: str, param_key: str = "params") -> str:
    """{param_key: state_dict} with CPU tensors and no 'module.' prefix (base_model.py:215-225)."""
    sd = OrderedDict()
    for k, v in _bare(net).state_dict().items():
        sd[k[7:] if k.startswith("module.") else k] = v.detach().cpu()
    torch.save({param_key: sd}, path)
    return path


def load_network(net, path: str, strict: bool = True, param_key: Optional[str] = "params"):
    """base_model.py:262-287: read the file, select param_key (None = the root dict), strip 'module.', load."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    sd = obj[param_key] if param_key is not None else obj
    sd = OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())
    return _bare(net).load_state_dict(sd, strict=strict)


def network_filename(models_dir: str, net_label: str, current_iter: int) -> str:
    """f'{net_label}_{iter}.pth', iter -1 -> 'latest' (base_model.py:205-208)."""
    return os.path.join(models_dir, f"{net_label}_{'latest' if current_iter == -1 else current_iter}.pth")


# ---------------------------------------------------------------------------------------------- optimizer state
def _param_slices(net: NAFNet):
    """(index, key, entry) in the reference parameter order (every NAFNet parameter is trainable)."""
    return [(i, k, net.entries[k]) for i, k in enumerate(net.ref_order)]


def adamw_state_dict(trainer) -> Dict:
    """The fused AdamW state of an NBPTrainer as torch.optim.AdamW.state_dict() over the reference parameters."""
    net: NAFNet = trainer.net
    state = {}
    step = torch.tensor(float(trainer.t))
    for i, k, e in _param_slices(net):
        state[i] = {"step": step.clone(),
                    "exp_avg": net._to_reference(e, trainer.exp_avg[e.offset:e.offset + e.numel]).detach().cpu(),
                    "exp_avg_sq": net._to_reference(e, trainer.exp_avg_sq[e.offset:e.offset + e.numel]).detach().cpu()}
    lr = _last_lr(trainer)
    group = {"lr": float(lr), "betas": tuple(float(b) for b in trainer.betas), "eps": float(trainer.eps),
             "weight_decay": float(trainer.wd), "amsgrad": False, "foreach": None, "maximize": False,
             "capturable": False, "differentiable": False, "fused": None, "initial_lr": float(trainer.lr),
             "params": [i for i, _, _ in _param_slices(net)]}
    return {"state": state, "param_groups": [group]}


def load_adamw_state_dict(trainer, sd: Dict) -> None:
    """Inverse of adamw_state_dict: per-parameter exp_avg / exp_avg_sq (reference layout) into the flat buffers."""
    net: NAFNet = trainer.net
    slices = _param_slices(net)
    if len(sd["param_groups"]) != 1 or len(sd["param_groups"][0]["params"]) != len(slices):
        raise ValueError("optimizer state does not match this network's parameters")
    steps = set()
    with torch.no_grad():
        for i, k, e in slices:
            st = sd["state"].get(i)
            if st is None:  # parameter never stepped
                trainer.exp_avg[e.offset:e.offset + e.numel] = 0
                trainer.exp_avg_sq[e.offset:e.offset + e.numel] = 0
                continue
            for name, buf in (("exp_avg", trainer.exp_avg), ("exp_avg_sq", trainer.exp_avg_sq)):
                v = st[name]
                if tuple(v.shape) != e.ref_shape:
                    raise ValueError(f"optimizer state {name} of {k}: shape {tuple(v.shape)} != {e.ref_shape}")
                buf[e.offset:e.offset + e.numel] = net._to_internal(e, v.to(torch.float32)).to(buf.device)
            steps.add(int(float(st["step"])))
    if len(steps) > 1:
        raise ValueError(f"per-parameter AdamW steps differ ({sorted(steps)}): the fused optimizer has one step count")
    g = sd["param_groups"][0]
    trainer.t = steps.pop() if steps else 0
    trainer.betas = tuple(g["betas"])
    trainer.eps, trainer.wd = float(g["eps"]), float(g["weight_decay"])
    trainer.lr = float(g.get("initial_lr", g["lr"]))


def _last_lr(trainer) -> float:
    """The lr the last iteration ran with: base_model.update_learning_rate (:164-174) steps the scheduler only from
    iteration 2 on, so after N iterations it has stepped N - 1 times (last_epoch = N - 1)."""
    s = trainer.scheduler
    return float(s(max(trainer.iter - 1, 0))) if s is not None else float(trainer.lr)


def scheduler_state_dict(trainer) -> Dict:
    """The TrueCosineAnnealingLR state in torch CosineAnnealingLR.state_dict() form after trainer.iter iterations of
    the reference loop: constructed (last_epoch 0, _step_count 1), then stepped once per iteration after the first."""
    s = trainer.scheduler
    it = max(trainer.iter - 1, 0)
    return {"T_max": s.T if s is not None else 0, "eta_min": s.eta_min if s is not None else 0.0,
            "base_lrs": [s.base if s is not None else trainer.lr], "last_epoch": it, "_step_count": it + 1,
            "verbose": False, "_get_lr_called_within_step": False, "_last_lr": [_last_lr(trainer)]}


def scaler_state_dict(trainer) -> Optional[Dict]:
    """torch.amp.GradScaler.state_dict() form of the trainer's device-side loss scaler (None without one)."""
    if trainer.scaler is None:
        return None
    sc = trainer.scaler.cpu()
    return {"scale": float(sc[0]), "growth_factor": float(sc[1]), "backoff_factor": float(sc[2]),
            "growth_interval": int(sc[3]), "_growth_tracker": int(trainer.ctl[1].item())}


def save_training_state(trainer, epoch: int, current_iter: int, states_dir: str) -> Optional[str]:
    """f'{iter}.state' = {'epoch', 'iter', 'optimizers': [AdamW state], 'schedulers': [...]} (base_model.py:290-314);
    nothing is written for current_iter == -1, as in the reference."""
    if current_iter == -1:
        return None
    state = {"epoch": int(epoch), "iter": int(current_iter), "optimizers": [adamw_state_dict(trainer)],
             "schedulers": [scheduler_state_dict(trainer)]}
    amp = scaler_state_dict(trainer)
    if amp is not None:  # base_model.py:309-310
        state["amp_scaler"] = amp
    path = os.path.join(states_dir, f"{current_iter}.state")
    torch.save(state, path)
    return path


def resume_training(trainer, resume_state) -> Dict:
    """base_model.py:316-333: restore the optimizer (and the scheduler position) from a training-state dict or file.
    Returns the dict (its 'epoch' / 'iter' are for the caller's loop)."""
    if isinstance(resume_state, str):
        resume_state = torch.load(resume_state, map_location="cpu", weights_only=True)
    opts, scheds = resume_state["optimizers"], resume_state["schedulers"]
    if len(opts) != 1:
        raise AssertionError("Wrong lengths of optimizers")
    load_adamw_state_dict(trainer, opts[0])
    if scheds and trainer.scheduler is not None:
        s = scheds[0]
        trainer.scheduler.T = s.get("T_max", trainer.scheduler.T)
        trainer.scheduler.eta_min = s.get("eta_min", trainer.scheduler.eta_min)
        trainer.scheduler.base = s.get("base_lrs", [trainer.scheduler.base])[0]
    if scheds:  # the iteration the scheduler stands at (see scheduler_state_dict)
        trainer.iter = int(scheds[0].get("last_epoch", 0)) + 1
    amp = resume_state.get("amp_scaler")
    if amp is not None and trainer.scaler is not None:  # base_model.py:332-333
        trainer.scaler.copy_(torch.tensor([amp["scale"], amp["growth_factor"], amp["backoff_factor"],
                                           float(amp["growth_interval"])]))
        trainer.ctl[1] = int(amp["_growth_tracker"])
        # the current upstream gradients carry the old scale: re-derive them from the restored one (other batch
        # sizes' buffers are refreshed when the trainer switches to them)
        trainer._refresh_up()
    return resume_state
