"""The union of the trace launches' intervals (csrc/hg_interval.h), the divisor of bench.py's roofline frac
(hg_counters.trace_busy_ms).  ADVICE r03: the old loop seeded its run with lo = 0, hi = -1, so a launch starting before
the reference launch (a negative offset) was merged into a run from 0 and the union came out short.  Compiled with g++
against a Python restatement; needs no GPU."""
import random
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HDR = ROOT / "halogen-pathtracer_amd" / "csrc" / "hg_interval.h"

DRIVER = r'''
#include "hg_interval.h"
#include <cstdio>
int main() {
    int n;
    while (std::scanf("%d", &n) == 1) {
        std::vector<std::pair<double, double>> iv(n);
        for (auto& x : iv) std::scanf("%lf %lf", &x.first, &x.second);
        std::printf("%.9f\n", hg_interval_union(iv));
    }
}
'''


def union_py(iv):
    """Length of the union: sweep over the sorted endpoints."""
    total, cur_lo, cur_hi = 0.0, None, None
    for a, b in sorted(iv):
        if cur_hi is None or a > cur_hi:
            if cur_hi is not None:
                total += cur_hi - cur_lo
            cur_lo, cur_hi = a, b
        else:
            cur_hi = max(cur_hi, b)
    return total + (cur_hi - cur_lo if cur_hi is not None else 0.0)


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("iv")
    (d / "main.cpp").write_text(DRIVER)
    exe = d / "iv"
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{HDR.parent}", str(d / "main.cpp"), "-o", str(exe)], check=True)
    return exe


def run(exe, cases):
    text = "".join(f"{len(iv)} " + " ".join(f"{a!r} {b!r}" for a, b in iv) + "\n" for iv in cases)
    out = subprocess.run([str(exe)], input=text, capture_output=True, text=True, check=True).stdout.split()
    return [float(x) for x in out]


def test_interval_union_negative_first_offset(driver):
    # the reference launch (offset 0) started 1.5 ms after another one: the union is 2.0 + 1.5, not 2.0
    cases = [[(0.0, 2.0), (-1.5, 1.0)], [(0.0, 1.0), (-3.0, -2.0)], [(-2.0, -1.0)], [], [(0.0, 0.0)],
             [(0.0, 1.0), (1.0, 2.0)], [(0.0, 5.0), (1.0, 2.0), (-1.0, 0.5)]]
    got = run(driver, cases)
    want = [3.5, 2.0, 1.0, 0.0, 0.0, 2.0, 6.0]
    assert got == pytest.approx(want, abs=1e-9)


def test_interval_union_random(driver):
    rng = random.Random(4)
    cases = []
    for _ in range(300):
        n = rng.randint(1, 12)
        iv = []
        for _ in range(n):
            a = rng.uniform(-20, 20)
            iv.append((a, a + rng.uniform(0, 8)))
        cases.append(iv)
    assert run(driver, cases) == pytest.approx([union_py(iv) for iv in cases], abs=1e-6)
