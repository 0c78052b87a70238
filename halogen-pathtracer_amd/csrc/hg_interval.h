// hg_interval.h — the union of the trace launches' [start, end) intervals (ms), the roofline's device time per launch
// (hg_counters.trace_busy_ms).  Launches on the trace streams overlap, and the offsets are taken relative to one of
// them (not necessarily the first to start), so an interval may begin at a negative offset.  Host-only and
// dependency-free: tests/test_interval_union.py compiles it with g++.
#pragma once
#include <algorithm>
#include <utility>
#include <vector>

inline double hg_interval_union(std::vector<std::pair<double, double>> iv) {
    if (iv.empty()) return 0.0;
    std::sort(iv.begin(), iv.end());
    double covered = 0.0, lo = iv.front().first, hi = iv.front().first;  // seeded from the earliest start
    for (const auto& x : iv) {
        if (x.first > hi) {  // a gap: close the current run
            covered += hi - lo;
            lo = x.first;
            hi = x.second;
        } else if (x.second > hi) {
            hi = x.second;
        }
    }
    return covered + (hi - lo);
}
