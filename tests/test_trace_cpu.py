"""roctx ranges (include/aac_trace.h, multi_agent_aac_amd/trace.py): the C ABI nests and unnests
ranges without a profiler attached, and the Python ranges are no-ops unless enabled."""
import contextlib


def test_trace_abi_nesting(native_lib):
    from multi_agent_aac_amd import trace
    L = trace._lib()
    d0 = L.aac_trace_push(b"outer")          # roctx: the pushed range's 0-based level
    d1 = L.aac_trace_push(b"inner")
    assert d0 >= 0 and d1 == d0 + 1
    L.aac_trace_mark(b"mark")
    assert L.aac_trace_pop() == d1            # the level of the range just closed
    assert L.aac_trace_pop() == d0


def test_ranges_off_by_default_and_on_when_enabled(native_lib):
    from multi_agent_aac_amd import trace
    was = trace.ENABLED
    try:
        trace.enable(False)
        assert isinstance(trace.range("x"), contextlib.nullcontext)
        trace.enable(True)
        r = trace.range("env_step")
        assert not isinstance(r, contextlib.nullcontext)
        with r:
            with trace.range("update.seg0"):
                trace.mark("m")
    finally:
        trace.enable(was)
