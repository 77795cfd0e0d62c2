"""Compare-exchange networks of rgc_device.h (make_cmpnet: Batcher odd-even merge sort,
pruned for the middle elements) against std::sort on random inputs with many ties, compiled
for the host with hipcc (the device code uses the same constexpr tables; no GPU call)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "repic-copy_amd", "csrc")

PROG = r"""
#include <algorithm>
#include <cstdio>
#include <random>
#include "rgc_device.h"
template <int N, typename T> int check(std::mt19937& g) {
  int bad = 0;
  for (int t = 0; t < 5000; ++t) {
    T v[N], w[N], u[N];
    for (int i = 0; i < N; ++i) v[i] = w[i] = u[i] = (T)(g() % 5);
    std::sort(w, w + N);
    rgc::cmpnet_apply<N, false>(v);
    rgc::mid_n<N>(u);
    for (int i = 0; i < N; ++i) bad += v[i] != w[i];
    bad += u[N / 2] != w[N / 2];
    if (N % 2 == 0) bad += u[N / 2 - 1] != w[N / 2 - 1];
  }
  return bad;
}
int main() {
  std::mt19937 g(7);
  int b = check<2, double>(g) + check<3, double>(g) + check<5, double>(g) + check<6, double>(g) +
          check<8, int>(g) + check<10, double>(g) + check<10, float>(g) + check<15, double>(g) +
          check<21, float>(g) + check<28, double>(g) + check<28, float>(g) + check<7, int>(g);
  std::printf("%d\n", b);
  return b != 0;
}
"""


HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")
def test_cmpnet_sorts_and_medians_match_std_sort(tmp_path):
    src = tmp_path / "net.hip"
    src.write_text(PROG)
    exe = tmp_path / "net"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-I" + CSRC, str(src),
                    "-o", str(exe)], check=True, capture_output=True, timeout=240)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout + r.stderr
