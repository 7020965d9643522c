"""gvx_imu_series_from_to -- host logic of the C ABI, no device -- against the
oracle (oracle/ins.c; MISC::getImuSeriesFromTo, misc.cc:330-384): bit-exact."""
import numpy as np
import pytest

import gvx
import oracle as orc
from gvx import synth_ba


def _imu():
    return synth_ba.make_imu_segment(np.random.default_rng(21), 120, t0=50.0)


@pytest.mark.parametrize("o0,o1", [(0.002, 0.0031), (0.00003, 0.00003), (0.00499, 0.00499), (0.0, 0.0),
                                   (0.002, 0.00499), (0.00003, 0.0)])
def test_series_matches_oracle(o0, o1):
    imu = _imu()
    t0, t1 = float(imu[10]["time"]) + o0, float(imu[60]["time"]) + o1
    a, b = gvx.imu_series_from_to(imu, t0, t1), orc.imu_series_from_to(imu, t0, t1)
    assert a is not None and b is not None and len(a) == len(b)
    for k in a.dtype.names:
        assert np.array_equal(a[k], b[k]), k
    assert a[-1]["time"] == t1


def test_series_outside_window():
    imu = _imu()
    t0 = float(imu[10]["time"])
    assert gvx.imu_series_from_to(imu, t0, float(imu[-1]["time"]) + 1.0) is None
    assert gvx.imu_series_from_to(imu, float(imu[0]["time"]) - 1.0, t0) is None
    assert gvx.imu_series_from_to(imu[:0], 0.0, 1.0) is None
