"""Drop-in overlay: run the reference's UNCHANGED train.py (and its pipeline engine, checkpoint
init, utils) with the decoder-layer hot path on picotron_amd's gfx950 kernels.

    PYTHONPATH=<this repo>/dropin:<picotron checkout> torchrun ... train.py --config cfg.json

`import picotron` then finds this package first.  It registers picotron_amd's hot-path modules under
the reference's module names -- the SAME module objects, so module globals such as
`picotron.process_group_manager.process_group_manager` are shared by the reference's own callers
(utils.py, checkpoint.py, pipeline_parallel/) and by picotron_amd -- and extends the package path to
the checkout's picotron/ directory for every module it does not replace (utils, checkpoint, data,
pipeline_parallel).  Nothing is copied from the checkout; nothing in it is modified.

Replaced (reference path -> module object):
    picotron/model.py                              picotron_amd.model
    picotron/process_group_manager.py              picotron_amd.process_group_manager
    picotron/tensor_parallel/{tensor_parallel,tp_communications}.py
    picotron/context_parallel/{context_parallel,cp_communications}.py
    picotron/data_parallel/{data_parallel,bucket}.py
    picotron/pipeline_parallel/pp_communications.py   picotron_amd.pipeline_parallel.pp_communications
                                                   (the PipelineParallel engine itself stays the checkout's)
"""
import importlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(os.path.dirname(_HERE))
if _REPO not in sys.path:
    sys.path.insert(0, _REPO)

REPLACED = ("process_group_manager", "model",
            "tensor_parallel", "tensor_parallel.tensor_parallel", "tensor_parallel.tp_communications",
            "context_parallel", "context_parallel.context_parallel", "context_parallel.cp_communications",
            "data_parallel", "data_parallel.data_parallel", "data_parallel.bucket",
            "pipeline_parallel.pp_communications")


def _checkout_dir():
    """The reference checkout's picotron/ directory: $PICOTRON_REFERENCE, else the next `picotron`
    directory on sys.path after this overlay."""
    env = os.environ.get("PICOTRON_REFERENCE")
    if env:
        cand = os.path.join(env, "picotron")
        return cand if os.path.isdir(cand) else None
    for entry in sys.path:
        cand = os.path.abspath(os.path.join(entry or os.getcwd(), "picotron"))
        if os.path.isdir(cand) and cand != _HERE:
            return cand
    return None


_ref = _checkout_dir()
if _ref is not None:
    __path__.append(_ref)

for _name in REPLACED:
    _mod = importlib.import_module("picotron_amd." + _name)
    sys.modules[__name__ + "." + _name] = _mod
    _parent, _, _leaf = (__name__ + "." + _name).rpartition(".")
    if _parent in sys.modules:   # picotron.pipeline_parallel (the checkout's) is not imported here:
        setattr(sys.modules[_parent], _leaf, _mod)   # its `from ...pp_communications import` finds ours
