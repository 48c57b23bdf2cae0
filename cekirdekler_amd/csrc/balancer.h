// Iterative heterogeneous load balancer — the reference's law, reproduced
// exactly (HelperFunctions.cs:190-280 loadBalance; history shift/average
// HelperFunctions.cs:119-156; per-compute-id state Cores.cs:544-613,
// :1065-1130).  Kept as a pure function so it is unit-testable and so every
// rank of a distributed job computes the identical split from the same
// exchanged timings.
#pragma once
#include <cstdint>
#include <vector>

namespace cek {

struct BalancerState {
  std::vector<long long> ranges;      // work-items per device
  std::vector<long long> references;  // absolute start per device
  std::vector<std::vector<double>> history;  // [depth][devices], oldest first
  std::vector<double> bench;          // last measured ms per device
  long long calls = 0;
  long long global_range = 0;
  long long local_range = 0;
  long long global_offset = 0;
};

constexpr int kHistoryDepth = 10;     // Cores.cs:1065 performanceHistoryDepth

// One application of the law.  Mutates `ranges` and `history` in place.
//   bench:  per-device milliseconds of the previous call for this id
//   smooth: moving-average smoothing (active once the oldest slot is filled)
//   total:  global range; step: quantisation (localRange or localRange*blobs)
void load_balance(const std::vector<double>& bench, bool smooth,
                  std::vector<std::vector<double>>& history, long long total,
                  std::vector<long long>& ranges, long long step);

// First-call split (Cores.cs:569-596): equal share, remainder to device 0,
// followed by load_balance with every benchmark = 10.
void initial_split(int devices, bool smooth, std::vector<std::vector<double>>& history,
                   long long total, std::vector<long long>& ranges, long long step);

}  // namespace cek
