"""The GPU inline-CRC scheme restated on the host (tests/crc_math_check.cpp):
per-chunk raw CRCs from the lane tables, shifted to the payload's end, the
end-aligned edge chunks and the metadata-checksum delta, against the
byte-serial crc32 / crc32_legacy of liberasurecode (upstream
src/utils/chksum/crc32.c; pyeclib core.py:59-63 -> pyeclib_c.c:248).  CPU
only: g++ on the harness and pyeclib_amd/csrc/crc32.cpp."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_chunk_crc_scheme_matches_serial_crc(tmp_path):
    exe = tmp_path / "crc_math_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "pyeclib_amd", "csrc"),
                    os.path.join(ROOT, "tests", "crc_math_check.cpp"),
                    os.path.join(ROOT, "pyeclib_amd", "csrc", "crc32.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failures" in out.stdout
