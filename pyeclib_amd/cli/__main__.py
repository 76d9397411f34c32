"""Entry point: ``python -m pyeclib_amd.cli`` (reference cli/__main__.py)."""
from __future__ import annotations

import argparse
import sys
from typing import NoReturn, Optional

from . import bench, check, verify, version
from . import list as list_cmd


def main(argv: Optional[list[str]] = None) -> NoReturn:
    parser = argparse.ArgumentParser(prog="pyeclib-backend",
                                     description="tool to get various erasure coding information")
    parser.add_argument("-V", "--version", action="store_const", dest="func",
                        const=version.version_command, help=version.DESCRIPTION)
    sub = parser.add_subparsers()
    commands = [("version", version, None), ("list", list_cmd, list_cmd.add_list_args),
                ("check", check, check.add_check_args),
                ("verify", verify, verify.add_verify_args),
                ("bench", bench, bench.add_bench_args)]
    for name, module, add_args in commands:
        p = sub.add_parser(name, help=module.DESCRIPTION)
        p.set_defaults(func=getattr(module, f"{name}_command"))
        if add_args is not None:
            add_args(p)
    args = parser.parse_args(argv)
    if args.func is None:
        parser.error("the following arguments are required: {%s}" % ",".join(sub.choices))
    sys.exit(args.func(args))


if __name__ == "__main__":
    main()
