"""`verify`: decode (or reconstruct) every combination of available
fragments, or a random sample of them (reference cli/verify.py:41-153).
Exit status 3 if any result was corrupt, 1 if any combination failed."""
from __future__ import annotations

import argparse
import itertools
import os
import random

from .. import api
from . import add_instance_args, expand_ec_types, make_driver, report_unusable

DESCRIPTION = "validate reconstructability of EC schemas"


def add_verify_args(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("-q", "--quiet", action="store_true")
    parser.add_argument("--reconstruct", "-r", action="store_true")
    parser.add_argument("-i", "--iterations", type=int, default=None)
    add_instance_args(parser)


def fragment_subsets(frags, keep, iterations):
    if iterations is None:
        return itertools.combinations(frags, keep)
    return (random.sample(frags, keep) for _ in range(iterations))


def check_instance(instance, reconstruct, frags, unavailable, data, iterations):
    """(combinations, failures, corrupt) over subsets of len(frags) - unavailable."""
    combinations = failures = corrupt = 0
    for subset in fragment_subsets(frags, len(frags) - unavailable, iterations):
        targets = [i for i, f in enumerate(frags) if f not in subset] if reconstruct else [None]
        for index in targets:
            combinations += 1
            try:
                if index is None:
                    ok = instance.decode(subset) == data
                else:
                    ok = instance.reconstruct(subset, [index])[0] == frags[index]
            except api.ECDriverError:
                failures += 1
                continue
            corrupt += not ok
    return combinations, failures, corrupt


def verify_command(args: argparse.Namespace) -> int:
    types = expand_ec_types(args.ec_type)
    data = os.urandom(args.segment_size)
    width = max(len(t) for t in types)
    if "isa_l_rs_lrc" in types:
        print(f"Using {args.n_data} data + {args.n_parity} parity (of which "
              f"{args.local_parity} may be local) with {args.unavailable} unavailable frags")
    else:
        print(f"Using {args.n_data} data + {args.n_parity} parity with "
              f"{args.unavailable} unavailable frags")
    any_failures = any_corrupt = 0
    for ec_type in types:
        if report_unusable(ec_type, width):
            continue
        try:
            instance = make_driver(ec_type, args)
        except api.ECDriverError:
            print(f"{ec_type:<{width}} could not be instantiated")
            continue
        frags = instance.encode(data)
        combinations, failures, corrupt = check_instance(
            instance, args.reconstruct, frags, args.unavailable, data, args.iterations)
        any_failures += failures
        any_corrupt += corrupt
        if corrupt:
            print(f"\x1b[91;40m{ec_type:<{width}} {combinations=}, {failures=}, {corrupt=}\x1b[0m")
        elif failures and not (args.reconstruct and failures < combinations):
            print(f"\x1b[1;91m{ec_type:<{width}} {combinations=}, {failures=}\x1b[0m")
        elif failures:
            print(f"{ec_type:<{width}} {combinations=}, {failures=}")
        else:
            print(f"{ec_type:<{width}} {combinations=}")
    return 3 if any_corrupt else 1 if any_failures else 0
