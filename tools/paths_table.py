#!/usr/bin/env python3
"""DESIGN.md §4.6's table from a tools/bench_paths.py --out JSON file: one
markdown row per case (kernel-clock median, fraction of 8 TB/s), with the
fresh-object, tiled and index-free columns where the case has them.

    python tools/paths_table.py profiles/r04_paths_final.json
"""
import json
import sys

LABELS = {
    "quad_dword_16M": ("Quad 16 B, 16M", "DWORD"),
    "quad_tile_16M": ("Quad forced onto TILE", "TILE"),
    "number_body_16M": ("Number 4 B (configs[1] body)", "DWORD x4"),
    "all_kinds_17B_16M": ("all 6 fixed kinds, 17 B", "rec"),
    "square_request_53B_16M": ("Calculator.square request 53 B", "TILE / rec unpack"),
    "square_response_19B_16M": ("Calculator.square response 19 B", "TILE / rec unpack"),
    "add_request_58B_16M": ("add request 58 B", "TILE / rec unpack"),
    "subtract_request_63B_16M": ("subtract / multiply request 63 B", "TILE / rec unpack"),
    "two_numbers_response_23B_16M": ("TwoNumbers response 23 B", "TILE / rec unpack"),
    "quad_aos_16M": ("Quad as 24-B structs (vtable slot)", "AoS run"),
    "quad_aos_plain_16M": ("Quad as plain 16-B structs", "AoS tile copy"),
    "all_kinds_aos_16M": ("all 6 kinds as 32-B structs (vtable slot)", "AoS layout pack / piece unpack"),
    "multiple_primitives_str0-64_4M": ("multiple_primitives, strings 0-64 B, 4M", "VAR"),
    "string_0-1024_1M": ("one string 0-1024 B, 1M", "VAR"),
    "string_0-16_8M": ("one string 0-16 B, 8M", "VAR"),
    "string_0-32_4M": ("one string 0-32 B, 4M", "VAR"),
    "two_str_request_0-32_4M": ("two strings + request envelope, 0-32 B, 4M", "VAR"),
}


def main(path):
    rows = json.load(open(path))
    print("| case | path | pack | unpack | also |")
    print("|---|---|---|---|---|")
    for r in rows:
        name, kind = LABELS.get(r["case"], (r["case"], r["path"]))
        also = []
        if "unpack_fill_us" in r:
            also.append(f'fresh objects {r["unpack_fill_us"]:.1f} us, {r["unpack_fill_frac"]:.2f}')
        if "unpack_tiled_us" in r:
            also.append(f'tiled unpack {r["unpack_tiled_us"]:.1f} us, {r["unpack_tiled_frac"]:.2f}')
        if "stream_us" in r:
            also.append(f'no index {r["stream_us"]:.1f} us, {r["stream_frac"]:.2f}')
        if not r["parity_ok"]:
            also.append("PARITY FAILED")
        print(f'| {name} | {kind} | {r["pack_us"]:.1f} us, {r["pack_frac"]:.2f} | '
              f'{r["unpack_us"]:.1f} us, {r["unpack_frac"]:.2f} | {"; ".join(also)} |')


if __name__ == "__main__":
    main(sys.argv[1])
