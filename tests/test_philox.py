"""Philox4x32-10 (csrc/philox.h) against the Random123 known-answer vectors, on the host."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import PKG
from philox_ref import philox4x32_10, test_philox_known_answer  # noqa: F401  (collected here)

HARNESS = r"""
#include <stdio.h>
#include "philox.h"
int main() {
  mppi_u4 c = {0, 0, 0, 0};
  mppi_u4 r = philox4x32_10(c, 0, 0);
  mppi_u4 c2 = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  mppi_u4 r2 = philox4x32_10(c2, 0xFFFFFFFFu, 0xFFFFFFFFu);
  mppi_u4 c3 = {7, 11, 3, 2};
  mppi_u4 r3 = philox4x32_10(c3, 12345u, 0u);
  printf("%08x %08x %08x %08x\n%08x %08x %08x %08x\n%u %u %u %u\n", r.x, r.y, r.z, r.w, r2.x, r2.y, r2.z, r2.w,
         r3.x, r3.y, r3.z, r3.w);
  return 0;
}
"""


def test_product_philox_header_matches_known_answers():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "h.cpp")
        open(src, "w").write(HARNESS)
        exe = os.path.join(d, "h")
        r = subprocess.run(["g++", "-O2", "-I", os.path.join(PKG, "csrc"), src, "-o", exe], capture_output=True,
                           text=True)
        if r.returncode != 0:
            pytest.fail(r.stderr)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    assert out[0] == "6627e8d5 e169c58d bc57ac4c 9b00dbd8"
    assert out[1] == "408f276d 41c83b0e a20bc7c6 6d5451fd"
    assert [int(v) for v in out[2].split()] == [int(v) for v in philox4x32_10(7, 11, 3, 2, 12345, 0)]
