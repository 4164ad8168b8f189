/* aac_trace.h -- roctx ranges around the hot path's host-side stages (SURVEY.md section 5 "Tracing").
 *
 * Replaces the reference's wall-clock brackets of the training loop (ATT/main:224-226 episode
 * reset, :260-279 choose_action + env.step, :436-447 update_myown) with ranges a profiler sees on the
 * same timeline as the kernels: `rocprofv3 --marker-trace` records them (rocprofiler-sdk roctx).
 * The Python side (multi_agent_aac_amd/trace.py) brackets the env step, replay push, auto-reset,
 * each captured update-graph segment replay and each gradient all-reduce. */
#ifndef AAC_TRACE_H
#define AAC_TRACE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Opens a nested range named `name` on the calling thread; returns its 0-based level (< 0: error). */
int aac_trace_push(const char *name);
/* Closes the innermost open range of the calling thread; returns its level (< 0: none was open). */
int aac_trace_pop(void);
/* An instantaneous marker. */
void aac_trace_mark(const char *name);
#ifdef __cplusplus
}
#endif
#endif /* AAC_TRACE_H */
