#!/usr/bin/env python3
"""Merge GEMM autotuner caches: later files override earlier ones per shape key.
usage: python tools/merge_tuning.py OUT IN1 [IN2 ...]"""
import json
import sys


def main():
    out, ins = sys.argv[1], sys.argv[2:]
    merged = {}
    for p in ins:
        for e in json.load(open(p)):
            k, v = e.rsplit("=", 1)
            merged[k] = v
    with open(out, "w") as f:
        json.dump([f"{k}={v}" for k, v in merged.items()], f, indent=0)
    print(f"{len(merged)} entries -> {out}")


if __name__ == "__main__":
    main()
