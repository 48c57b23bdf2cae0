#include "balancer.h"

#include <algorithm>
#include <numeric>

namespace cek {

static size_t argmax(const std::vector<long long>& v) {
  // first maximum, as Functions.maxIndex
  size_t best = 0;
  for (size_t i = 1; i < v.size(); ++i)
    if (v[i] > v[best]) best = i;
  return best;
}

void load_balance(const std::vector<double>& bench, bool smooth,
                  std::vector<std::vector<double>>& history, long long total,
                  std::vector<long long>& ranges, long long step) {
  const size_t n = ranges.size();
  if (n == 0) return;
  if (step <= 0) step = 1;
  std::vector<double> thr(n, 0.0);
  std::vector<long long> tmp(n, 0);
  double total_bench = 0.01 * static_cast<double>(n);
  for (double b : bench) total_bench += b;
  double total_thr = 0;
  for (size_t i = 0; i < n; ++i) {
    thr[i] = (total_bench / (bench[i] + 0.01)) * static_cast<double>(ranges[i] + 1);
    total_thr += thr[i];
  }
  if (total_thr <= 0.0000001) total_thr = 0.01;

  std::vector<double> norm(n, 0.0);
  if (smooth) {
    for (size_t i = 0; i < n; ++i) norm[i] = thr[i] / total_thr;
    // shift one step older, newest last (performanceHistoryShiftOld)
    for (size_t d = 0; d + 1 < history.size(); ++d) history[d] = history[d + 1];
    if (!history.empty()) history.back() = norm;
    // average (performanceHistoryAverage)
    std::vector<double> avg(n, 0.0);
    for (auto& h : history)
      for (size_t i = 0; i < n; ++i) avg[i] += h[i];
    double div = 1.0 / static_cast<double>(history.size());
    for (size_t i = 0; i < n; ++i) avg[i] *= div;
    norm = avg;
  }
  const bool use_hist = smooth && !history.empty() && history[0][0] > 0.00001;
  for (size_t i = 0; i < n; ++i) {
    double p = use_hist ? norm[i] : thr[i] / total_thr;
    if (ranges[i] != 0) {
      tmp[i] = ranges[i] -
               static_cast<long long>(static_cast<double>(ranges[i] - static_cast<double>(total) * p) * 0.3);
    } else {
      tmp[i] = static_cast<long long>(static_cast<double>(total) *
                                      (total_bench / (bench[i] + 0.01)) / total_thr);
    }
  }
  for (size_t i = 0; i < n; ++i) {
    long long rem = tmp[i] % step;
    if (rem < step / 2)
      ranges[i] = tmp[i] - rem;
    else
      ranges[i] = tmp[i] + (step - rem);
  }
  auto sum = [&]() { return std::accumulate(ranges.begin(), ranges.end(), 0LL); };
  while (sum() > total) ranges[argmax(ranges)] -= step;
  while (sum() < total) ranges[argmax(ranges)] += step;
}

void initial_split(int devices, bool smooth, std::vector<std::vector<double>>& history,
                   long long total, std::vector<long long>& ranges, long long step) {
  ranges.assign(devices, 0);
  long long acc = 0;
  for (int i = 0; i < devices; ++i) {
    ranges[i] = total / devices;
    acc += ranges[i];
  }
  if (acc != total) ranges[0] += total - acc;
  std::vector<double> init(devices, 10.0);
  load_balance(init, smooth, history, total, ranges, step);
}

}  // namespace cek
