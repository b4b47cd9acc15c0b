"""Python facade over sa::StereoAlgorithm (stereoalgorithms_amd/algorithm.py): the failure paths that Initialize
reports before touching a GPU (reference RAFTStereoAlgorithm.cpp:37-40: the calibration file must exist)."""
import pytest

from stereoalgorithms_amd import _native as N


@pytest.mark.skipif(not N.available(), reason="native library not built")
def test_missing_calibration_is_an_error(tmp_path):
    from stereoalgorithms_amd.algorithm import StereoAlgorithm
    with pytest.raises(RuntimeError, match="calibration file not found"):
        StereoAlgorithm("raftstereo-realtime", str(tmp_path / "nope.yml"))


@pytest.mark.skipif(not N.available(), reason="native library not built")
def test_unparsable_calibration_is_an_error(tmp_path):
    from stereoalgorithms_amd.algorithm import StereoAlgorithm
    bad = tmp_path / "bad.yml"
    bad.write_text("this is not an OpenCV FileStorage file\n")
    with pytest.raises(RuntimeError, match="calibration"):
        StereoAlgorithm("raftstereo-realtime", str(bad))
