"""Timing events that can be recorded inside a captured HIP graph.

``torch.cuda.Event(external=True)`` is refused on ROCm ("External events are
disallowed in rocm"), so a graph replay could only be timed as a whole.  HIP
itself records an event inside stream capture as an external event node when
it is recorded with ``hipEventRecordWithFlags(..., hipEventRecordExternal)``;
:class:`GraphEvent` does that through the HIP runtime torch has loaded (one
runtime per process, see :mod:`lens_amd.native`).  Used by
``Colony.capture(timing=True)``: the kernel times of replayed steps (bench
kinetics / diffusion split) without a Python-issued eager step.

Measurement plumbing only: nothing on the simulation path depends on it.
"""

from __future__ import annotations

import ctypes

_HIP = None
HIP_EVENT_RECORD_EXTERNAL = 0x01


def _hip():
    global _HIP
    if _HIP is None:
        import torch  # noqa: F401  -- the runtime torch loaded (SONAME libamdhip64.so.7)
        lib = ctypes.CDLL('libamdhip64.so.7')
        lib.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        lib.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _HIP = lib
    return _HIP


class GraphEvent:
    """A timing HIP event; ``record()`` on a capturing stream becomes an event
    node of the graph, re-recorded at every replay."""

    def __init__(self):
        h = ctypes.c_void_p()
        rc = _hip().hipEventCreate(ctypes.byref(h))
        if rc != 0:
            raise RuntimeError('hipEventCreate failed (%d)' % rc)
        self._h = h

    def record(self, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _hip().hipEventRecordWithFlags(self._h, ctypes.c_void_p(s.cuda_stream), HIP_EVENT_RECORD_EXTERNAL)
        if rc != 0:
            raise RuntimeError('hipEventRecordWithFlags failed (%d)' % rc)

    def elapsed_time(self, end: 'GraphEvent') -> float:
        ms = ctypes.c_float()
        rc = _hip().hipEventElapsedTime(ctypes.byref(ms), self._h, end._h)
        if rc != 0:
            raise RuntimeError('hipEventElapsedTime failed (%d)' % rc)
        return float(ms.value)

    def __del__(self):
        try:
            if self._h and _HIP is not None:
                _HIP.hipEventDestroy(self._h)
        except Exception:
            pass
