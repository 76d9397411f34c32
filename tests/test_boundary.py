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
