// Host-side runtime probes (see probe.cpp).
#pragma once
#include "common.h"

namespace cek {

struct LaunchRate {
  int threads = 0, launches = 0;
  double host_ms = 0, drain_ms = 0, launches_per_s = 0;
  std::vector<double> per_thread_ms;
};

// T threads, each on its own stream of device `ordinal`, launch `kernel`
// (from `code_object`, the runtime ABI: two pointers + offset + size) with
// one 64-thread work-group `launches` times; host time until every launch
// call returned, and until the device drained.
LaunchRate launch_rate_probe(int ordinal, const std::string& code_object, const std::string& kernel, int threads,
                             int launches, int mode = 0);

}  // namespace cek
