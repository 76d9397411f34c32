"""The drop-in boundary, checked on CPU: pyeclib's own C extension compiles,
unmodified, against include/erasurecode_amd.h in place of
<liberasurecode/erasurecode.h> (src/pyeclib_c/pyeclib_c.c:34), and every
liberasurecode_* symbol it references is exported by libpyeclib_amd.so.
That is the claim of INTEGRATION.md §3: linking pyeclib_c against this
library instead of -lerasurecode (pyproject.toml:46-51) needs no source change.

The reference tree exists only in the build container; on a machine without
it (the GPU box) the test is skipped.  It only compiles the reference file
(object code, never linked or run) -- nothing of it is copied into the repo.
"""
import os
import re
import shutil
import subprocess
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_C = "/root/reference/src/pyeclib_c/pyeclib_c.c"
LIB = os.path.join(ROOT, "pyeclib_amd", "libpyeclib_amd.so")


def _nm(*args):
    return subprocess.run(["nm", *args], capture_output=True, text=True, check=True).stdout


@pytest.mark.skipif(not os.path.exists(REF_C), reason="reference tree not present")
@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("nm") is None,
                    reason="gcc/nm missing")
def test_pyeclib_c_compiles_against_our_header_and_links_symbols(tmp_path):
    pyinc = sysconfig.get_paths()["include"]
    if not os.path.exists(os.path.join(pyinc, "Python.h")):
        pytest.skip("Python.h not installed")
    shim = tmp_path / "inc" / "liberasurecode"
    shim.mkdir(parents=True)
    (shim / "erasurecode.h").write_text(
        f'#include "{os.path.join(ROOT, "include", "erasurecode_amd.h")}"\n')
    obj = tmp_path / "pyeclib_c.o"
    r = subprocess.run(["gcc", "-c", "-fPIC", "-O1", "-Wall", "-Werror=implicit-function-declaration",
                        f"-I{tmp_path / 'inc'}", f"-I{pyinc}",
                        f"-I{os.path.dirname(REF_C)}", REF_C, "-o", str(obj)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    needed = set(re.findall(r"\bU (liberasurecode_\w+)", _nm("-u", str(obj))))
    assert len(needed) >= 14, needed
    exported = set(re.findall(r"\bT (\w+)", _nm("-D", "--defined-only", LIB)))
    missing = needed - exported
    assert not missing, f"pyeclib_c.c needs symbols libpyeclib_amd.so lacks: {missing}"


@pytest.mark.skipif(shutil.which("nm") is None or shutil.which("strings") is None,
                    reason="nm/strings missing")
def test_product_library_has_no_ab_switches():
    """The product library carries no tuning or probe switches (round-3
    verdict): the memory-only probes that write wrong parity
    (ECAMD_ENC_NOCOMP / ECAMD_DEC_NOCOMP) and every other launch switch exist
    only in the A/B build (`make -C pyeclib_amd/csrc ab`), and the launch
    path reads no environment variable -- the runtime's knobs, which only
    choose between identical outputs, are read once per instance."""
    text = subprocess.run(["strings", "-a", LIB], capture_output=True, text=True,
                          check=True).stdout
    for name in ("ECAMD_ENC_NOCOMP", "ECAMD_DEC_NOCOMP", "ECAMD_ENC_CH", "ECAMD_ENC_NTL",
                 "ECAMD_ENC_NB", "ECAMD_DEC_NB", "ECAMD_EDGE_SIDE", "ECAMD_DATA_COPY",
                 "ECAMD_ENC_PER_CU", "ECAMD_DEC_PER_CU", "ECAMD_REC_PER_CU",
                 "ECAMD_CRC_PER_CU", "ECAMD_CRC_NTL", "ECAMD_XCD", "ECAMD_ENC_R3",
                 "ECAMD_DEC_R3", "ECAMD_CRC_STREAM", "ECAMD_CRC_V", "ECAMD_CRC_R", "ECAMD_REC_CRC_FREE"):
        assert name not in text, f"{name} is in the product library"
    exported = set(re.findall(r"\bT (\w+)", _nm("-D", "--defined-only", LIB)))
    assert "ecamd_ab_set" not in exported
    # the kept runtime knobs are read in one place (Knobs::from_env)
    src = open(os.path.join(ROOT, "pyeclib_amd", "csrc", "ec_runtime.cpp")).read()
    assert src.count("std::getenv") == 3, "getenv outside env_on / env_long / legacy CRC"
    impl = open(os.path.join(ROOT, "pyeclib_amd", "csrc", "ec_kernels_impl.hpp")).read()
    assert "getenv" not in impl
