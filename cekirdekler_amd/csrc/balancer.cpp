#include "balancer.h"

#include <algorithm>
#include <cmath>
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

static void quantize_fix(std::vector<long long>& ranges, const std::vector<double>& target, long long total,
                         long long step) {
  const size_t n = ranges.size();
  for (size_t i = 0; i < n; ++i) {
    long long t = static_cast<long long>(std::max(0.0, target[i]));
    long long rem = t % step;
    ranges[i] = rem < step / 2 ? t - rem : t + (step - rem);
  }
  auto sum = [&]() { return std::accumulate(ranges.begin(), ranges.end(), 0LL); };
  while (sum() > total) ranges[argmax(ranges)] -= step;
  while (sum() < total) ranges[argmax(ranges)] += step;
}

bool predict_split(FitState& fs, const std::vector<double>& bench, double wall_ms, long long total,
                   std::vector<long long>& ranges, long long step, bool warm) {
  const size_t n = ranges.size();
  if (n == 0) return false;
  if (step <= 0) step = 1;
  if (fs.samples.size() != n) {
    fs.samples.assign(n, {});
    fs.single_wall.assign(n, -1.0);
    fs.probed.assign(n, 0);
  }
  // 1) record this compute: a sample per computing device, keyed by range
  //    (a repeated range refreshes its time: an EWMA, so old noise fades)
  int active = 0, alone = -1;
  double tmax = 0;
  std::vector<char> mask(n, 0);
  for (size_t i = 0; i < n; ++i) mask[i] = ranges[i] > 0;
  if (fs.last_active.size() == n && fs.last_active != mask) warm = false;  // a switch call
  fs.last_active = mask;
  for (size_t i = 0; i < n; ++i) {
    if (ranges[i] <= 0 || i >= bench.size() || bench[i] <= 0) continue;
    ++active;
    alone = static_cast<int>(i);
    tmax = std::max(tmax, bench[i]);
    if (!warm) continue;
    auto& v = fs.samples[i];
    const double r = static_cast<double>(ranges[i]);
    auto it = std::find_if(v.begin(), v.end(), [&](const std::pair<double, double>& p) {
      return std::abs(p.first - r) <= 0.01 * r;
    });
    if (it != v.end()) {
      it->second = 0.5 * it->second + 0.5 * bench[i];
    } else {
      v.emplace_back(r, bench[i]);
      if (static_cast<int>(v.size()) > kFitSamples) v.erase(v.begin());
    }
  }
  // the configuration that chose the recorded call's split: the law, or
  // the predictor (a fitted split, a single device, a probe)
  const bool by_law = fs.decision == "law";
  bool settled = fs.prev_ranges.size() == n;
  for (size_t i = 0; settled && i < n; ++i)
    settled = std::llabs(ranges[i] - fs.prev_ranges[i]) * 100 <= total;
  fs.prev_ranges = ranges;
  if (by_law) fs.law_ranges = ranges;
  // hand back to the law: from its own last split when another
  // configuration ran the recorded call
  auto to_law = [&]() {
    fs.decision = "law";
    if (by_law || fs.law_ranges.size() != n) return false;
    ranges = fs.law_ranges;
    return true;
  };
  if (warm && active > 0 && wall_ms > 0 && by_law) {
    fs.law_settled = settled ? fs.law_settled + 1 : 0;
    // the median of the last settled law calls: what the law does now (an
    // average over every settled call would keep the slow first ones — a
    // host-resident stream's first calls are several times slower — and a
    // minimum keeps one lucky call)
    if (fs.law_settled >= 3) {
      fs.law_walls.push_back(wall_ms);
      if (static_cast<int>(fs.law_walls.size()) > kLawWalls) fs.law_walls.erase(fs.law_walls.begin());
      std::vector<double> v = fs.law_walls;
      std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
      fs.law_wall = v[v.size() / 2];
    }
    if (active >= 2) {
      const double ov = std::max(0.0, wall_ms - tmax);
      fs.o_multi = fs.o_multi < 0 ? ov : 0.7 * fs.o_multi + 0.3 * ov;
    }
  } else if (warm && active > 0 && wall_ms > 0) {
    if (active >= 2) {
      const double ov = std::max(0.0, wall_ms - tmax);
      fs.o_multi = fs.o_multi < 0 ? ov : 0.7 * fs.o_multi + 0.3 * ov;
      fs.multi_wall = fs.multi_wall < 0 ? wall_ms : 0.5 * fs.multi_wall + 0.5 * wall_ms;
    } else if (fs.recording_probe && alone == fs.probe_dev) {
      fs.probe_walls.push_back(wall_ms);
    } else {
      double& w = fs.single_wall[alone];
      w = w < 0 ? wall_ms : 0.5 * w + 0.5 * wall_ms;
    }
  }
  if (fs.probe_left == 0 && !fs.probe_walls.empty() && fs.probe_dev >= 0) {  // probe over
    const auto& v = fs.probe_walls;
    fs.single_wall[fs.probe_dev] = *std::min_element(v.begin(), v.end());
    fs.probe_walls.clear();
  }
  fs.recording_probe = false;
  // 2) fits t = a + b·r (least squares over distinct ranges)
  fs.a.assign(n, 0.0);
  fs.b.assign(n, 0.0);
  for (size_t i = 0; i < n; ++i) {
    const auto& v = fs.samples[i];
    if (v.size() < 2) {
      return to_law();
    }
    double sx = 0, sy = 0, sxx = 0, sxy = 0;
    for (auto& p : v) {
      sx += p.first;
      sy += p.second;
      sxx += p.first * p.first;
      sxy += p.first * p.second;
    }
    const double k = static_cast<double>(v.size());
    const double den = k * sxx - sx * sx;
    if (den <= 0) {
      return to_law();
    }
    double b = (k * sxy - sx * sy) / den;
    double a = (sy - b * sx) / k;
    if (b <= 0) {  // flat or noisy: all fixed cost, a tiny slope keeps the split defined
      a = sy / k;
      b = 1e-9 * std::max(a, 1e-6);
    }
    if (a < 0) {  // proportional: refit through the origin
      a = 0;
      b = sxy / sxx;
    }
    fs.a[i] = a;
    fs.b[i] = b;
  }
  // 3) water-filling: equal predicted finish time T over the devices kept
  std::vector<char> keep(n, 1);
  double T = 0;
  for (;;) {
    double inv = 0, ab = 0;
    for (size_t i = 0; i < n; ++i)
      if (keep[i]) {
        inv += 1.0 / fs.b[i];
        ab += fs.a[i] / fs.b[i];
      }
    T = (static_cast<double>(total) + ab) / inv;
    // drop the device with the largest fixed cost whose share is under a step
    int drop = -1;
    for (size_t i = 0; i < n; ++i)
      if (keep[i] && (T - fs.a[i]) / fs.b[i] < static_cast<double>(step) &&
          (drop < 0 || fs.a[i] > fs.a[drop]))
        drop = static_cast<int>(i);
    if (drop < 0) break;
    keep[drop] = 0;
  }
  int kept = 0;
  for (char c : keep) kept += c;
  size_t best = 0;  // the best single device by its fit
  for (size_t i = 1; i < n; ++i)
    if (fs.a[i] + fs.b[i] * total < fs.a[best] + fs.b[best] * total) best = i;
  const double pred_multi = T + std::max(0.0, fs.o_multi);
  fs.predicted_multi_ms = pred_multi;
  // 4) single device or split: the single device's MEASURED wall time against
  //    the split's predicted one (a probe measures it, once)
  bool single = kept < 2;
  if (!single) {
    if (fs.probe_left > 0) {
      single = true;
      best = static_cast<size_t>(fs.probe_dev);
    } else if (fs.single_wall[best] < 0) {
      const double guess = fs.a[best] + fs.b[best] * static_cast<double>(total);
      if (!fs.probed[best] && guess <= kProbeGate * pred_multi) {
        fs.probed[best] = 1;
        fs.probe_left = kProbeCalls;
        fs.probe_dev = static_cast<int>(best);
        single = true;
      }
    } else {
      single = fs.single_wall[best] <= std::max(pred_multi, fs.multi_wall);
    }
  }
  // the guard: defer to the law until its settled split is timed, and
  // whenever the chosen configuration has been measured no faster than it
  // (a probe still runs to completion: it is the measurement)
  if (fs.probe_left == 0) {
    const double cand = single ? fs.single_wall[best] : fs.multi_wall;
    if (fs.law_wall < 0 || (cand > 0 && cand >= kGuardMargin * fs.law_wall)) return to_law();
  }
  std::vector<double> target(n, 0.0);
  if (single) {
    target[best] = static_cast<double>(total);
    fs.decision = fs.probe_left > 0 ? "probe" : "single";
    if (fs.probe_left > 0) {
      --fs.probe_left;
      fs.recording_probe = true;
    }
  } else {
    for (size_t i = 0; i < n; ++i)
      if (keep[i]) target[i] = (T - fs.a[i]) / fs.b[i];
    fs.decision = "multi";
  }
  quantize_fix(ranges, target, total, step);
  return true;
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
