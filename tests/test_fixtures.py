"""MNN's tensor fixture text format (niti_amd.fixtures): reading as
`stream >> v` does (testModel.cpp:43-56), writing as expressDemo's output.txt, checkFile's
comparison, and the C4 / NHWC element orders of the reference's own fixture files (slices committed
under tests/golden/ by make_fixture_slices.py; the whole files are read when /root/reference is
present)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
from niti_amd import fixtures as F  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference/execution-engine/resource/model"


def test_squeezenet_c4_slice_layout():
    # the first image row of SqueezeNet's input: C4 [1][1][1][227][4], three channels + a zero lane
    a = F.read_txt(os.path.join(GOLD, "squeezenet_input_row0.txt"), 227 * 4, np.int16)
    x = F.c4_to_nchw(a, 1, 3, 1, 227)
    assert x.shape == (1, 3, 1, 227)
    assert np.all(a.reshape(227, 4)[:, 3] == 0)  # the pad lane
    assert x[0, :, 0, 0].tolist() == [-54, -58, -97]
    assert np.array_equal(F.nchw_to_c4(x).reshape(-1), a)


def test_mobilenet_nhwc_slice_layout():
    a = F.read_txt(os.path.join(GOLD, "mobilenet_qnt_input_row0.txt"), 224 * 3, np.uint8)
    x = F.nhwc_to_nchw(a, 1, 3, 1, 224)
    assert x[0, :, 0, 0].tolist() == [62, 62, 62] and x[0, :, 0, 1].tolist() == [45, 48, 46]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_fixture_files_whole():
    sq = F.read_txt(f"{REF}/SqueezeNet/input.txt", dtype=np.float32)
    assert sq.size == 227 * 227 * 4 and np.all(sq.reshape(-1, 4)[:, 3] == 0)
    mb = F.read_txt(f"{REF}/MobileNet/qnt_input.txt", 224 * 224 * 3, np.uint8)
    assert mb.size == 224 * 224 * 3
    # flt_input.txt opens with a stray '>>>' line: `stream >> v` fails at once and leaves the
    # tensor unread, and read_txt stops there the same way (asking for the tensor's count raises)
    assert F.read_txt(f"{REF}/MobileNet/flt_input.txt").size == 0
    with pytest.raises(ValueError):
        F.read_txt(f"{REF}/MobileNet/flt_input.txt", 224 * 224 * 3)


def test_write_read_check_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    x = rng.integers(-127, 128, (2, 5, 3, 4)).astype(np.int8)
    p1, p2 = str(tmp_path / "a.txt"), str(tmp_path / "b.txt")
    F.write_txt(p1, F.nchw_to_c4(x))
    back = F.c4_to_nchw(F.read_txt(p1, dtype=np.int8), 2, 5, 3, 4)
    assert np.array_equal(back, x)
    y = x.astype(np.float32).reshape(-1).copy()
    y[7] += 0.5
    F.write_txt(p2, F.nchw_to_c4(y.reshape(x.shape)))
    bad = F.check_file(p1, p2, 0.1)
    assert len(bad) == 1 and bad[0][2] - bad[0][1] == pytest.approx(0.5)
    assert F.check_file(p1, p2, 1.0) == []
    with pytest.raises(ValueError):
        F.read_txt(p1, count=F.nchw_to_c4(x).size + 1)
    with pytest.raises(ValueError):
        F.read_txt(p2, dtype=np.int8)  # 0.5 does not fit int8
