"""roctx ranges named after the reference's ``torch.profiler.record_function`` labels
(temporalpoints.py:421-653, pointwarper.py:217-241), so a ``rocprofv3 --marker-trace`` timeline
of a frame lines up with a profile of the reference stage by stage.

The fused kernels cover several reference stages each; a fused stage opens the nest of the
labels it replaces (e.g. the neighbour-MLP kernel: ``feat_net`` > ``densitynet`` > ``rgbnet``),
so every reference label appears, with the extent of the kernel that computes it. Host-side only:
inside a HIP graph replay nothing is emitted (bench.py's stage timings come from eager frames,
where the ranges are). Without a profiler attached the calls are no-ops in the library."""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")
_lib = None
_tried = False

# fused stage -> reference labels it replaces (outermost first)
STAGES = {
    "skeleton": ("poc_fre", "forward_warp", "transform_net", "calc_rec_abs_T"),
    "lbs": ("weighted_G_tw",),
    "sampling": ("sample_ray",),
    "knn": ("knn", "knn-post"),
    "mlp": ("feat_net", "densitynet", "rgbnet"),
    "composite": ("pre-mask", "Alphas2Weights", "post-mask", "segment_coo"),
}


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("APN_ROCTX", "1") == "0":
        return None
    roots = [os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib"), ""]
    for name in _LIBS:
        for root in roots:
            try:
                lib = ctypes.CDLL(os.path.join(root, name) if root else name)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            _lib = lib
            return _lib
    return None


def available() -> bool:
    return _load() is not None


def begin(name: str):
    """Open the nested ranges of fused stage ``name`` (close them with end(name))."""
    lib = _load()
    if lib is not None:
        for lab in STAGES[name]:
            lib.roctxRangePushA(lab.encode())


def end(name: str):
    lib = _load()
    if lib is not None:
        for _ in STAGES[name]:
            lib.roctxRangePop()


class Sequence:
    """Consecutive stages of one call: ``switch(name)`` closes the open stage's ranges and opens
    the next one's (``switch(None)`` only closes); leaving the ``with`` block -- normally or by an
    exception raised between two switches -- closes whatever is still open, so a failed call never
    leaves pushed ranges behind for later markers to nest under."""

    def __init__(self):
        self._open = None

    def switch(self, name):
        if self._open is not None:
            end(self._open)
        self._open = name
        if name is not None:
            begin(name)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.switch(None)
        return False


@contextlib.contextmanager
def stage(name: str):
    """Nested roctx ranges of the reference labels that fused stage ``name`` replaces."""
    begin(name)
    try:
        yield
    finally:
        end(name)
