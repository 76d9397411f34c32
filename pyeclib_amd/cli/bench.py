"""`bench`: encode / decode MB/s of each scheme through ECDriver, the
reference tool's own throughput definition (reference cli/bench.py:40-99:
MB = iterations x segment_size / 2^20 over wall time, one object per call)."""
from __future__ import annotations

import argparse
import os
import random
import time

from .. import api
from . import add_instance_args, expand_ec_types, make_driver, report_unusable

DESCRIPTION = "benchmark EC schemas"


def add_bench_args(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("-e", "--encode", action="store_true")
    parser.add_argument("-d", "--decode", action="store_true")
    add_instance_args(parser, default_segment_size=2**20)
    parser.add_argument("--iterations", "-i", type=int, default=200)


def _rate(iterations: int, segment_size: int, seconds: float) -> str:
    return f"{iterations * segment_size / 2**20 / seconds:.1f}MB/s"


def bench_command(args: argparse.Namespace) -> None:
    types = expand_ec_types(args.ec_type)
    data = os.urandom(args.segment_size + args.iterations)
    width = max(len(t) for t in types)
    k, u = args.n_data, args.unavailable
    print(f"Using {k} data + {args.n_parity} parity with {u} unavailable frags")
    run_encode = args.encode or not args.decode
    run_decode = args.decode or not args.encode
    for ec_type in types:
        if report_unusable(ec_type, width):
            continue
        try:
            instance = make_driver(ec_type, args)
        except api.ECDriverError:
            print(f"{ec_type:<{width}} could not be instantiated")
            continue
        frags = instance.encode(data[:args.segment_size])
        if run_encode:
            t0 = time.time()
            for i in range(args.iterations):
                instance.encode(data[i:i + args.segment_size])
            print(f"{ec_type} (encode): {_rate(args.iterations, args.segment_size, time.time() - t0)}")
        if run_decode:
            t0 = time.time()
            for _ in range(args.iterations):
                # u data fragments unavailable, replaced by as many parity fragments
                # (flat XOR: all parity; LRC: local parity share extra)
                chosen = random.sample(frags[:k], k - u)
                if ec_type.startswith("flat_xor"):
                    chosen += frags[k:]
                elif ec_type == "isa_l_rs_lrc":
                    chosen += random.sample(frags[k:], u + args.local_parity - 1)
                else:
                    chosen += random.sample(frags[k:], u)
                instance.decode(chosen)
            print(f"{ec_type} (decode): {_rate(args.iterations, args.segment_size, time.time() - t0)}")
