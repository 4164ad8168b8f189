// aac_trace.cpp -- include/aac_trace.h over rocprofiler-sdk's roctx (what `rocprofv3 --marker-trace`
// records).  Host code only; with no profiler attached a range is a few nanoseconds.
#include <rocprofiler-sdk-roctx/roctx.h>

#include "../../include/aac_trace.h"

extern "C" int aac_trace_push(const char *name) { return name ? roctxRangePushA(name) : -1; }

extern "C" int aac_trace_pop(void) { return roctxRangePop(); }

extern "C" void aac_trace_mark(const char *name) {
    if (name) roctxMarkA(name);
}
