// roctx ranges around the device library's phases (visible in rocprofv3 --marker-trace and in
// profiler timelines); free when no tool is attached.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace svm355 {

struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace svm355
