"""`pyeclib-backend`-style command line for the MI355X backend.

Same subcommands, options, output lines and exit codes as the reference tool
(src/pyeclib/cli/__main__.py:36-80: version, list, check, verify, bench),
answered from this package's ECDriver, ALL_EC_TYPES and VALID_EC_TYPES.
Run as ``python -m pyeclib_amd.cli <subcommand>``.
"""
from __future__ import annotations

import argparse
from typing import Iterable

from .. import api

# abbreviation -> ec_type prefix (reference cli/__init__.py:29-40)
ABBREVIATIONS = {
    "all": "", "isa-l": "isa_l_", "isa_l": "isa_l_", "isal": "isa_l_",
    "jerasure": "jerasure_", "flat-xor": "flat_xor_", "flat_xor": "flat_xor_",
    "flatxor": "flat_xor_", "xor": "flat_xor_",
}


def expand_ec_types(user_types: Iterable[str] | None) -> list[str]:
    """Replace abbreviations by the ec_types they stand for; sorted, unique."""
    names = set(user_types or ["all"])
    for abbrev in [a for a in names if a in ABBREVIATIONS]:
        names.discard(abbrev)
        prefix = ABBREVIATIONS[abbrev]
        names.update(t for t in api.ALL_EC_TYPES if t.startswith(prefix))
    return sorted(names)


def add_instance_args(parser: argparse.ArgumentParser, default_segment_size: int = 1024) -> None:
    """Scheme options shared by verify and bench (reference cli/__init__.py:56-104)."""
    parser.add_argument("--ec-type", action="append", type=str)
    parser.add_argument("--n-data", "--ndata", "-k", metavar="K", type=int, default=10)
    parser.add_argument("--n-parity", "--nparity", "-m", metavar="M", type=int, default=5)
    parser.add_argument("--local-parity", "-l", metavar="L", type=int, default=2)
    parser.add_argument("--unavailable", "-u", metavar="N", type=int, default=2)
    parser.add_argument("--segment-size", "-s", metavar="BYTES", type=int,
                        default=default_segment_size)


def make_driver(ec_type: str, args: argparse.Namespace) -> api.ECDriver:
    return api.ECDriver(ec_type=ec_type, k=args.n_data, m=args.n_parity,
                        local_parity=args.local_parity)


def report_unusable(ec_type: str, width: int) -> bool:
    """Print why ec_type cannot be benchmarked / verified; True if it can't."""
    if ec_type not in api.ALL_EC_TYPES:
        print(f"{ec_type:<{width}} unknown")
        return True
    if ec_type not in api.VALID_EC_TYPES:
        print(f"{ec_type:<{width}} not available")
        return True
    return False
