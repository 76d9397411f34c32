"""The `pyeclib-backend` command line (python -m pyeclib_amd.cli), following
the reference's CLI tests (test/test_pyeclib_cli.py): output lines, statuses
and exit codes.  Availability is patched where the real answer depends on
whether a GPU is present."""
import io
import platform
import re
from contextlib import redirect_stderr, redirect_stdout

import pytest

from pyeclib_amd import api
from pyeclib_amd.cli.__main__ import main


def run(argv):
    out, err = io.StringIO(), io.StringIO()
    with redirect_stdout(out), redirect_stderr(err), pytest.raises(SystemExit) as caught:
        main(argv)
    return caught.value.code, out.getvalue(), err.getvalue()


@pytest.mark.parametrize("argv", [["version"], ["-V"]])
def test_version(argv):
    code, out, _ = run(argv)
    assert code is None and out.endswith("\n")
    parts = [line.split(" ", 1) for line in out[:-1].split("\n")]
    assert [p[0] for p in parts] == ["pyeclib", "liberasurecode", platform.python_implementation()]
    assert all(re.match(r"^\d+\.\d+\.\d+", p[1]) for p in parts)
    assert parts[1][1] == "1.8.0"


def test_list_all(monkeypatch):
    monkeypatch.setattr(api, "VALID_EC_TYPES", ["liberasurecode_rs_vand", "amd_rs_vand"])
    code, out, _ = run(["list"])
    rows = [line.split() for line in out[:-1].split("\n")]
    assert [r[0] for r in rows] == sorted(api.ALL_EC_TYPES)
    assert {r[1] for r in rows} == {"available", "missing"}
    assert dict(rows)["amd_rs_vand"] == "available" and code == 0


def test_list_none_available(monkeypatch):
    monkeypatch.setattr(api, "VALID_EC_TYPES", [])
    code, out, _ = run(["list", "liberasurecode_rs_vand"])
    assert out.split() == ["liberasurecode_rs_vand", "missing"] and code == 1


def test_list_unknown_and_mixed(monkeypatch):
    monkeypatch.setattr(api, "VALID_EC_TYPES", ["liberasurecode_rs_vand"])
    code, out, _ = run(["list", "missing-backend"])
    assert out.split() == ["missing-backend", "unknown"] and code == 1
    code, out, _ = run(["list", "missing-backend", "liberasurecode_rs_vand"])
    rows = [line.split() for line in out[:-1].split("\n")]
    assert rows == [["liberasurecode_rs_vand", "available"], ["missing-backend", "unknown"]]
    assert code == 0


def test_list_abbreviations(monkeypatch):
    monkeypatch.setattr(api, "VALID_EC_TYPES", ["isa_l_rs_cauchy", "isa_l_rs_vand"])
    code, out, _ = run(["list", "isal"])
    rows = [line.split() for line in out[:-1].split("\n")]
    assert [r[0] for r in rows] == sorted(t for t in api.ALL_EC_TYPES if t.startswith("isa_l_"))
    assert code == 0
    code, out, _ = run(["list", "--available", "flatxor"])
    assert out == "" and code == 1
    code, out, _ = run(["list", "--available"])
    assert out[:-1].split("\n") == ["isa_l_rs_cauchy", "isa_l_rs_vand"] and code == 0


def test_check(monkeypatch):
    code, _, err = run(["check"])
    assert code == 2 and "the following arguments are required: ec_type" in err
    monkeypatch.setattr(api, "VALID_EC_TYPES", ["liberasurecode_rs_vand"])
    assert run(["check", "liberasurecode_rs_vand"]) == (0, "liberasurecode_rs_vand is available\n", "")
    assert run(["check", "-q", "liberasurecode_rs_vand"]) == (0, "", "")
    monkeypatch.setattr(api, "VALID_EC_TYPES", [])
    assert run(["check", "liberasurecode_rs_vand"]) == (1, "liberasurecode_rs_vand is missing\n", "")
    assert run(["check", "--quiet", "liberasurecode_rs_vand"]) == (1, "", "")
    assert run(["check", "unknown-backend"]) == (2, "unknown-backend is unknown\n", "")
    assert run(["check", "-q", "unknown-backend"]) == (2, "", "")


def test_no_subcommand():
    code, _, err = run([])
    assert code == 2 and "the following arguments are required" in err


def test_verify_and_bench_skip_unavailable(monkeypatch):
    monkeypatch.setattr(api, "VALID_EC_TYPES", [])
    code, out, _ = run(["verify", "--ec-type", "amd_rs_vand", "--ec-type", "nope"])
    assert code == 0
    assert out.split("\n")[1:3] == ["amd_rs_vand not available", "nope        unknown"]
    code, out, _ = run(["bench", "--ec-type", "amd_rs_vand", "-i", "1"])
    assert "amd_rs_vand not available" in out


@pytest.mark.gpu
def test_verify_gpu_schemes():
    code, out, _ = run(["verify", "--ec-type", "amd_rs_vand", "--ec-type", "isal", "-k", "6",
                        "-m", "3", "-u", "3"])
    assert code == 0, out
    # "isal" expands to every isa_l_* type; lrc / vand_inv have no GPU backend
    for name in ("amd_rs_vand", "isa_l_rs_cauchy", "isa_l_rs_vand"):
        assert re.search(rf"^{name} +combinations=84$", out, re.M), out
    assert re.search(r"^isa_l_rs_lrc +not available$", out, re.M)
    code, out, _ = run(["verify", "-r", "--ec-type", "liberasurecode_rs_vand", "-k", "4", "-m",
                        "2", "-u", "2", "-i", "10"])
    assert code == 0 and "combinations=20" in out


@pytest.mark.gpu
def test_bench_gpu_schemes():
    code, out, _ = run(["bench", "--ec-type", "amd_rs_vand", "--ec-type", "isa_l_rs_cauchy",
                        "-k", "10", "-m", "4", "-i", "3", "-s", "65536"])
    assert code is None
    assert re.search(r"amd_rs_vand \(encode\): [\d.]+MB/s", out)
    assert re.search(r"isa_l_rs_cauchy \(decode\): [\d.]+MB/s", out)


@pytest.mark.gpu
def test_file_tools_roundtrip(tmp_path, oracle):
    """BASELINE configs[0]: k=4 m=2 liberasurecode_rs_vand, one 1 MiB file
    through tools/pyeclib_encode.py and tools/pyeclib_decode.py, 2 fragments
    dropped; fragments equal the oracle's."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "obj.bin"
    data = os.urandom(1 << 20)
    src.write_bytes(data)
    frag_dir = tmp_path / "frags"
    frag_dir.mkdir()
    subprocess.run([sys.executable, os.path.join(root, "tools", "pyeclib_encode.py"), "4", "2",
                    "0", "liberasurecode_rs_vand", str(tmp_path), "obj.bin", str(frag_dir)],
                   check=True, capture_output=True)
    frags = [(frag_dir / f"obj.bin.{i}").read_bytes() for i in range(6)]
    assert frags == oracle.encode(4, 2, data)
    subprocess.run([sys.executable, os.path.join(root, "tools", "pyeclib_decode.py"), "4", "2",
                    "0", "liberasurecode_rs_vand"]
                   + [str(frag_dir / f"obj.bin.{i}") for i in (0, 2, 4, 5)]
                   + [str(tmp_path / "out")], check=True, capture_output=True)
    assert (tmp_path / "out.decoded").read_bytes() == data
