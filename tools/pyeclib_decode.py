#!/usr/bin/env python3
"""Fragment files -> <filename>.decoded through pyeclib_amd.ECDriver.

Same positional interface as the reference's tools/pyeclib_decode.py:27-40
(k m l ec_type fragment... filename); BASELINE configs[0] harness.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyeclib_amd import ECDriver  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description="Decoder for PyECLib (MI355X backend).")
    ap.add_argument("k", type=int, help="number of data elements")
    ap.add_argument("m", type=int, help="number of parity elements")
    ap.add_argument("l", type=int, help="number of local parity elements", default=-1)
    ap.add_argument("ec_type", help="EC algorithm used")
    ap.add_argument("fragments", metavar="fragment", nargs="+", help="fragments to decode")
    ap.add_argument("filename", help="output file")
    args = ap.parse_args()
    print("k = %d, m = %d" % (args.k, args.m))
    print("ec_type = %s" % args.ec_type)
    print("fragments = %s" % args.fragments)
    print("filename = %s" % args.filename)
    driver = ECDriver(k=args.k, m=args.m, ec_type=args.ec_type, local_parity=args.l)
    fragments = []
    for path in args.fragments:
        with open(path, "rb") as fp:
            fragments.append(fp.read())
    with open("%s.decoded" % args.filename, "wb") as fp:
        fp.write(driver.decode(fragments))


if __name__ == "__main__":
    main()
