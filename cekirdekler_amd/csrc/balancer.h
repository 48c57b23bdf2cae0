// Iterative heterogeneous load balancer — the reference's law, reproduced
// exactly (HelperFunctions.cs:190-280 loadBalance; history shift/average
// HelperFunctions.cs:119-156; per-compute-id state Cores.cs:544-613,
// :1065-1130).  Kept as a pure function so it is unit-testable and so every
// rank of a distributed job computes the identical split from the same
// exchanged timings.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace cek {

// Opt-in overhead-aware predictor, in the slot the reference left for one
// (HelperFunctions.cs:163-178: PID / derivative predictors that return null).
// The reference law assumes time ∝ range, so a device with a large fixed
// cost per compute (launch + sync latency, host-thread fan-out) keeps a share
// that makes the compute slower than leaving it out.  The predictor fits
// t_i = a_i + b_i·r_i per device from the (range, time) samples of this
// compute id (warm calls only: the first computes of an id allocate and
// upload), splits by water-filling (equal predicted finish time; a device
// whose best share is below one step gets none) and predicts that split's
// wall time as T + the measured multi-device overhead (wall − slowest
// device).  The best single device is then run alone for a few calls, once,
// when its predicted time is within 50 % of that (kProbeGate), and then the
// configuration with the lower wall time is used: measured for the single
// device; for the split the larger of the prediction and the measured wall
// of recent split calls (a fit that misses a cost of co-execution — a CPU
// pool's wake-ups, contention on shared hardware — cannot keep choosing a
// split that is slower in fact).  Until every device has a fit, and until
// the law's own settled split has been timed, it defers to the law; and it
// never keeps a configuration whose measured wall time is not below the
// law's (so it can only be as slow as the law, or faster).
struct FitState {
  std::vector<std::vector<std::pair<double, double>>> samples;  // per device: (range, ms), distinct ranges
  double o_multi = -1;                 // EWMA of wall − max device ms over multi-device calls
  std::vector<double> single_wall;     // per device: EWMA wall ms of calls it ran alone (−1: never)
  std::vector<char> probed;
  int probe_left = 0, probe_dev = -1;
  bool recording_probe = false;        // the call being recorded ran as a probe
  std::vector<char> last_active;       // devices with a share in the last recorded call
  std::vector<double> probe_walls;     // the probe calls' wall ms, in order
  std::string decision = "law";        // law | multi | single | probe
  std::vector<double> a, b;            // last fits (ms, ms per work item)
  double predicted_multi_ms = 0;
  double multi_wall = -1;              // EWMA wall ms of recent fitted-split calls (−1: none yet)
  // Guard: the law's own split, measured once it has
  // settled (three calls in a row in which no device's range moved more
  // than 1 % of the total).  The predictor deviates from the law only after this is
  // known and only to a configuration not measured slower than it.
  double law_wall = -1;                // median wall ms of the last settled law calls (−1: not yet)
  std::vector<double> law_walls;       // the last kLawWalls settled law calls' wall ms
  int law_settled = 0;                 // consecutive settled law calls
  std::vector<long long> prev_ranges;  // the ranges of the previous recorded call
  // the last split the law chose: restored when the predictor hands back to
  // the law (the law cannot bring a device back from a zero range)
  std::vector<long long> law_ranges;
};

constexpr int kFitSamples = 8;
// the predictor keeps a configuration only while it is measured at least
// 3 % faster than the law's best settled call
constexpr double kGuardMargin = 0.97;
// settled law calls the guard's reference is the median of (a minimum kept
// one lucky call: a 0.023 ms wave frame against a typical 0.031 made the
// GPU alone, 0.027, look no faster than the law)
constexpr int kLawWalls = 5;
// The first compute after the set of devices with a share changed is not
// recorded: it pays the move (slices going up to their new device), a cost
// of the switch, not of the split.  A probe runs the best single device
// alone for kProbeCalls computes; its wall time is the minimum over the
// recorded ones.
constexpr int kProbeCalls = 3;
// The best single device is probed (once) when its fitted time alone is
// within this factor of the split's predicted time.  Its fit comes from
// calls it shared with the others, and sharing can slow a device a lot: a
// CPU device streaming host memory next to a GPU's DMA on the same memory
// measured 4.35 ms per range by its shared-call fit and 2.4-2.6 ms alone
// (hetero_stream, iters 1), so a tight gate never measures what it would save.
constexpr double kProbeGate = 1.5;

// Records the last compute of this id (its ranges, per-device ms and wall ms;
// `warm` = not one of the id's first computes) and, when every device has a
// fit, writes the next split into `ranges` (returns true); false = apply the
// reference law instead.
bool predict_split(FitState& fs, const std::vector<double>& bench, double wall_ms, long long total,
                   std::vector<long long>& ranges, long long step, bool warm = true);

struct BalancerState {
  std::vector<long long> ranges;      // work-items per device
  std::vector<long long> references;  // absolute start per device
  std::vector<std::vector<double>> history;  // [depth][devices], oldest first
  std::vector<double> bench;          // last measured ms per device
  long long calls = 0;
  long long global_range = 0;
  long long local_range = 0;
  long long global_offset = 0;
  double last_wall_ms = 0;  // wall time of the last compute of this id
  FitState fit;             // overhead-aware predictor (opt-in)
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
