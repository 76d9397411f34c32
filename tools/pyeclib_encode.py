#!/usr/bin/env python3
"""File -> k + m fragment files through pyeclib_amd.ECDriver.

Same positional interface as the reference's tools/pyeclib_encode.py:27-37
(k m l ec_type file_dir filename fragment_dir) and the same output names
(<fragment_dir>/<filename>.<i>); BASELINE configs[0] harness.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyeclib_amd import ECDriver  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description="Encoder for PyECLib (MI355X backend).")
    ap.add_argument("k", type=int, help="number of data elements")
    ap.add_argument("m", type=int, help="number of total parity elements")
    ap.add_argument("l", type=int, help="number of local parity elements", default=-1)
    ap.add_argument("ec_type", help="EC algorithm used")
    ap.add_argument("file_dir", help="directory with the file")
    ap.add_argument("filename", help="file to encode")
    ap.add_argument("fragment_dir", help="directory to drop encoded fragments")
    args = ap.parse_args()
    print("k = %d, m = %d" % (args.k, args.m))
    print("ec_type = %s" % args.ec_type)
    print("filename = %s" % args.filename)
    driver = ECDriver(k=args.k, m=args.m, ec_type=args.ec_type, local_parity=args.l)
    with open(os.path.join(args.file_dir, args.filename), "rb") as fp:
        payload = fp.read()
    for i, fragment in enumerate(driver.encode(payload)):
        with open("%s/%s.%d" % (args.fragment_dir, args.filename, i), "wb") as fp:
            fp.write(fragment)


if __name__ == "__main__":
    main()
