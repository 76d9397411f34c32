"""`check`: exit status 0 / 1 / 2 = available / missing / unknown."""
from __future__ import annotations

import argparse

from .. import api

DESCRIPTION = "check for backend availability"


def add_check_args(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("-q", "--quiet", action="store_true")
    parser.add_argument("ec_type")


def check_command(args: argparse.Namespace) -> int:
    if args.ec_type in api.VALID_EC_TYPES:
        status, code = "available", 0
    elif args.ec_type in api.ALL_EC_TYPES:
        status, code = "missing", 1
    else:
        status, code = "unknown", 2
    if not args.quiet:
        print(args.ec_type, "is", status)
    return code
