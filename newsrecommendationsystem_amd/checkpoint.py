"""Checkpoints in the reference's format (src/train.py:54-64,144-159,264-279;
src/evaluate.py:281-288).

A checkpoint is the dict torch.save writes at src/train.py:266-277:
  {'model_state_dict': NRMS.state_dict(), 'optimizer_state_dict':
   Adam.state_dict(), 'step': int, 'early_stop_value': -val_auc}
where early_stop_value is a numpy float64 (the negated AUC of evaluate()).
Module parameter names are the reference's (nrms.py), and HipAdam keeps
torch.optim.Adam's state keys and param_group fields, so files interchange
in both directions: a reference checkpoint resumes on the HIP path and a HIP
checkpoint resumes under the reference's train.py.

Loading never unpickles arbitrary objects: torch.load(weights_only=True) with
only numpy's scalar reconstruction allowed (the early_stop_value entry).
"""
import os

import numpy as np
import torch


def _safe_numpy_globals():
    try:
        from numpy._core.multiarray import scalar
    except ImportError:                       # numpy < 2
        from numpy.core.multiarray import scalar
    return [scalar, np.dtype, type(np.dtype(np.float64))]


def load(path, map_location="cpu"):
    """The checkpoint dict, read with torch.load(weights_only=True)."""
    with torch.serialization.safe_globals(_safe_numpy_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def latest_checkpoint(directory):
    """Path of the ckpt-{step}.pth with the largest step, or None
    (src/train.py:54-64)."""
    if not os.path.isdir(directory):
        return None
    found = {}
    for name in os.listdir(directory):
        try:
            found[int(name.split(".")[-2].split("-")[-1])] = name
        except (IndexError, ValueError):
            continue
    if not found:
        return None
    return os.path.join(directory, found[max(found)])


def resume(path, model, optimizer=None):
    """Load model (and optimizer) state as src/train.py:144-159 does; returns
    (step, early_stop_value). The model keeps its device: tensors are mapped
    onto it, and the optimizer's moments follow its parameters' devices.

    The file is read onto the CPU: load_state_dict copies the parameters onto
    the model's device, and Optimizer.load_state_dict moves exp_avg /
    exp_avg_sq to each parameter's device but leaves the 'step' counters where
    they were loaded -- on the CPU, as the reference keeps them (a CUDA step
    tensor would cost HipAdam a device-to-host sync per parameter per step)."""
    ck = load(path, map_location="cpu")
    model.load_state_dict(ck["model_state_dict"])
    if optimizer is not None:
        optimizer.load_state_dict(ck["optimizer_state_dict"])
        for st in optimizer.state.values():
            step = st.get("step")
            if torch.is_tensor(step) and step.device.type != "cpu":
                st["step"] = step.cpu()
    return int(ck["step"]), ck["early_stop_value"]


def save(path, model, optimizer, step, early_stop_value):
    """src/train.py:266-277."""
    torch.save({"model_state_dict": model.state_dict(),
                "optimizer_state_dict": optimizer.state_dict(),
                "step": int(step),
                "early_stop_value": np.float64(early_stop_value)}, path)
