"""Weights-only checkpoints.

The reference saves ``{'model_kwargs': model.get_kwargs(), 'model_state_dict': model.state_dict()}``
with ``torch.save`` and restores it with ``utils.load_model`` (lib/utils.py:519-523:
``model_class(**ckpt['model_kwargs'])`` + ``load_state_dict(strict=False)``). For TemporalPoints the
kwargs (temporalpoints.py:176-200) hold the stage-1 TiNeuVox *module* and numpy arrays, so that
file restores only through a full unpickle, which this package never does on a checkpoint.

Here the same two keys are kept with plain data only -- tensors, numbers, strings, lists, dicts --
so ``torch.load(path, weights_only=True)`` restores them; the TiNeuVox module becomes its
constructor kwargs plus its state dict:

    {'format': 'apn-weights-only-1', 'model_class': 'TemporalPoints' | 'TiNeuVox',
     'model_kwargs': {...}, 'model_state_dict': {...},
     'tineuvox_class': 'TiNeuVox' | 'TiNeuVoxHeads', 'tineuvox_kwargs': {...},
     'tineuvox_state_dict': {...}}            # TemporalPoints only

``to_weights_only`` converts a checkpoint dict in the reference layout (loaded where its classes
are importable and the file is trusted, e.g. the training machine) or this package's own models;
``load_model`` is the drop-in for lib/utils.py:519-523 on converted files."""
import numpy as np
import torch

FORMAT = "apn-weights-only-1"


def _plain(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().clone()
    if isinstance(v, np.ndarray):
        return torch.from_numpy(np.array(v))
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _plain(x) for k, x in v.items()}
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    raise TypeError(f"not plain checkpoint data: {type(v).__name__}")


def _state(sd):
    return {k: v.detach().cpu().clone() for k, v in sd.items()}


def to_weights_only(ckpt: dict) -> dict:
    """Reference-layout checkpoint dict -> weights-only dict. ``ckpt['model_kwargs']['tineuvox']``
    (TemporalPoints checkpoints) may be any module with ``get_kwargs()`` and ``state_dict()``:
    the reference TiNeuVox (tineuvox.py:180-199) or this package's TiNeuVox / TiNeuVoxHeads."""
    mk = dict(ckpt["model_kwargs"])
    out = {"format": FORMAT, "model_state_dict": _state(ckpt["model_state_dict"])}
    tnv = mk.pop("tineuvox", None)
    if tnv is not None:
        out["model_class"] = "TemporalPoints"
        out["tineuvox_class"] = "TiNeuVoxHeads" if type(tnv).__name__ == "TiNeuVoxHeads" else "TiNeuVox"
        out["tineuvox_kwargs"] = _plain(tnv.get_kwargs())
        out["tineuvox_state_dict"] = _state(tnv.state_dict())
    else:
        out["model_class"] = "TiNeuVox"
    out["model_kwargs"] = _plain(mk)
    return out


def checkpoint_of(model) -> dict:
    """The weights-only checkpoint of a TemporalPoints / TiNeuVox of this package."""
    return to_weights_only({"model_kwargs": model.get_kwargs(), "model_state_dict": model.state_dict()})


def save_checkpoint(model, path) -> None:
    torch.save(checkpoint_of(model), path)


def read_checkpoint(path) -> dict:
    """torch.load(weights_only=True): nothing in the file is executed; a reference-layout file
    (pickled TiNeuVox module, numpy arrays) is refused by the loader itself."""
    try:
        ck = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:   # the weights-only unpickler refuses anything but plain data
        raise ValueError(f"{path}: not a weights-only checkpoint ({type(e).__name__}); convert a reference "
                         "checkpoint with apn_amd.checkpoint.to_weights_only where its classes are importable") from e
    if not isinstance(ck, dict) or ck.get("format") != FORMAT:
        raise ValueError(f"{path}: not an {FORMAT} checkpoint")
    return ck


def build(ck: dict, device=None):
    """Model from a weights-only checkpoint dict: model_class(**model_kwargs) (TemporalPoints:
    with the TiNeuVox rebuilt from its kwargs and state dict), then load_state_dict(strict=False)
    as lib/utils.py:519-523."""
    from .tineuvox import TiNeuVox, TiNeuVoxHeads
    if ck.get("format") != FORMAT:
        raise ValueError(f"not an {FORMAT} checkpoint")
    if ck["model_class"] == "TiNeuVox":
        model = TiNeuVox(**ck["model_kwargs"])
    elif ck["model_class"] == "TemporalPoints":
        from .temporalpoints import TemporalPoints
        cls = TiNeuVoxHeads if ck["tineuvox_class"] == "TiNeuVoxHeads" else TiNeuVox
        tnv = cls(**ck["tineuvox_kwargs"])
        tnv.load_state_dict(ck["tineuvox_state_dict"], strict=False)
        model = TemporalPoints(**ck["model_kwargs"], tineuvox=tnv)
    else:
        raise ValueError(f"unknown model_class {ck['model_class']!r}")
    model.load_state_dict(ck["model_state_dict"], strict=False)
    return model.to(device) if device is not None else model


def load_checkpoint(path, device=None):
    return build(read_checkpoint(path), device)


def load_model(model_class, ckpt_path):
    """lib/utils.py:519-523 on a weights-only checkpoint (model_class must match the file's)."""
    ck = read_checkpoint(ckpt_path)
    if ck["model_class"] != model_class.__name__:
        raise ValueError(f"{ckpt_path} holds a {ck['model_class']}, not a {model_class.__name__}")
    return build(ck)
