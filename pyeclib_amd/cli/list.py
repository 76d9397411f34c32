"""`list`: availability of EC backends (reference cli/list.py)."""
from __future__ import annotations

import argparse

from .. import api
from . import expand_ec_types

DESCRIPTION = "list availability of EC backends"


def add_list_args(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("-a", "--available", action="store_true",
                        help="display only available backends")
    parser.add_argument("ec_type", nargs="*", type=str,
                        help="display these backends (default: all)")


def list_command(args: argparse.Namespace) -> int:
    names = expand_ec_types(args.ec_type)
    width = max(len(n) for n in names)
    available = 0
    for name in names:
        usable = name in api.VALID_EC_TYPES
        available += usable
        if args.available:
            if usable:
                print(name)
            continue
        status = ("available" if usable else "missing") if name in api.ALL_EC_TYPES else "unknown"
        print(f"{name:<{width}} {status}")
    return 0 if available else 1
