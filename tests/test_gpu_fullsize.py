"""Parity at BASELINE.json's full sizes (configs C2-C5, one GPU, data
resident in HBM), through properties that do not need the CPU oracle to
walk gigabytes:

* an independent restatement of the path in plain torch on the device:
  hyperslab box per chunk (``storage.py:95``), the mask of
  ``storage.py:126-153`` (``== _FillValue``, ``< valid_min``,
  ``> valid_max``, all in the variable dtype as bench.py passes them) and
  count/sum/min/max (``storage.py:98-100``); count, min and max must match
  bit for bit, the f32/f64 sum within the north star's 1e-6 relative;
* for the shuffled config (C4), the kernel on the byte-shuffled chunks must
  give what it gives on the same chunks stored unshuffled (count, min, max
  exact; the un-shuffle changes the summation order, so sum within 1e-6);
* additivity over a split of the chunk list: counts add, min/max of the
  halves are the min/max of the whole (exact), sums add within 1e-6.

The workloads are bench.py's CONFIGS (same generator, fill planting and
selection tables).  C4 holds 34 GB and C5 69 GB in HBM.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_full_size_config(gpu, name):
    """tests/_fullsize_check.py in a fresh process (torch initialises the GPU
    first there; this process already holds libpyas_hip's context)."""
    r = subprocess.run([sys.executable, "-u", "-m", "tests._fullsize_check", name], cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{name}: rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert f"fullsize {name} OK" in r.stdout
    print(r.stdout.strip())


@pytest.mark.parametrize("name", ["c4", "c5", "c4u", "c5u"])
def test_full_size_samples_against_oracle(gpu, name):
    """Real-size chunks of C4 (64 x 128^3 f32, shuffled, masked) and C5 (256 x
    32^3 f64, boundary-heavy hyperslab) against the oracle's storage.py and
    _from_storage combine (tests/_fullsize_oracle.py, fresh process); "u":
    the same configs without valid_max, chunks spread over the whole grid,
    so the sums at scale run over every element."""
    r = subprocess.run([sys.executable, "-u", "-m", "tests._fullsize_oracle", name], cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{name}: rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert f"fullsize-oracle {name} OK" in r.stdout
    print(r.stdout.strip())
