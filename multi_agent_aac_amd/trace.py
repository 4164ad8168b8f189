"""roctx ranges on the hot path (include/aac_trace.h; SURVEY.md section 5 "Tracing").

The reference brackets its loop with wall-clock prints (ATT/main:224-226, :260-279, :436-447).
Here the stages are roctx ranges that ``rocprofv3 --marker-trace`` puts on the kernel timeline:
``act``, ``env_step``, ``replay_push``, ``auto_reset``, ``update`` and, inside it, one
``update.seg<k>`` per captured graph segment and one ``allreduce`` per gradient collective.

Off unless ``AAC_ROCTX=1`` (a profiling run sets it): ``range`` is then a shared no-op object, so
the timed loop pays nothing for it.
"""
import contextlib
import os

ENABLED = os.environ.get("AAC_ROCTX", "0") == "1"
_NULL = contextlib.nullcontext()


class _Range:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name.encode()

    def __enter__(self):
        _lib().aac_trace_push(self.name)

    def __exit__(self, *exc):
        _lib().aac_trace_pop()
        return False


_L = None


def _lib():
    global _L
    if _L is None:
        import ctypes
        from . import _native
        _L = _native.lib()
        _L.aac_trace_push.argtypes = [ctypes.c_char_p]
        _L.aac_trace_pop.argtypes = []
        _L.aac_trace_mark.argtypes = [ctypes.c_char_p]
        _L.aac_trace_mark.restype = None
    return _L


def range(name):          # noqa: A001  (the roctx vocabulary)
    """Context manager: a roctx range named ``name`` when tracing is on, else a no-op."""
    return _Range(name) if ENABLED else _NULL


def mark(name):
    if ENABLED:
        _lib().aac_trace_mark(name.encode())


def enable(on=True):
    """Switch the ranges on / off in this process (tests, tools)."""
    global ENABLED
    ENABLED = bool(on)
