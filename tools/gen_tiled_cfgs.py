"""Regenerate csrc/hkt_cfg.h's configuration table and one instantiation file
per configuration (csrc/hkt_c<id>.hip) for K1 variant 5 (hk_tiled.h).
The first row for a given (N, value type) is the default tspgpu.cpp picks.

    python tools/gen_tiled_cfgs.py
"""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tsp-mpi-reduction_amd", "csrc")

# (id, value type, N, L, threads per workgroup, distance copies R, workgroups per CU)
CFGS = [
    (14, "double", 15, 10, 256, 1, 6),
    (20, "int32_t", 15, 10, 256, 1, 8),
    (22, "double", 14, 10, 256, 1, 6),
    (23, "double", 13, 10, 256, 1, 6),
    (12, "double", 15, 10, 256, 1, 5),
    (2, "double", 15, 11, 256, 1, 3),
    (0, "double", 15, 11, 512, 1, 2),
    (1, "double", 15, 10, 256, 1, 4),
    (3, "double", 15, 10, 512, 1, 2),
    (4, "double", 15, 11, 512, 2, 2),
    (5, "double", 14, 11, 512, 1, 2),
    (6, "double", 14, 10, 256, 1, 4),
    (7, "int32_t", 15, 11, 256, 1, 4),
    (8, "int32_t", 15, 11, 512, 1, 2),
    (9, "int32_t", 14, 11, 256, 1, 4),
    (10, "double", 13, 10, 256, 1, 4),
    (11, "double", 15, 10, 128, 1, 6),
    (13, "double", 15, 10, 192, 1, 5),
    (15, "double", 15, 9, 256, 1, 6),
    (16, "double", 15, 9, 256, 1, 7),
    (17, "double", 15, 10, 256, 2, 5),
    (18, "double", 15, 10, 256, 1, 7),
    (19, "int32_t", 15, 10, 256, 1, 6),
    (21, "int32_t", 15, 11, 256, 1, 5),
    (24, "int32_t", 14, 10, 256, 1, 6),
    (26, "double", 12, 10, 256, 1, 6),
    (25, "double", 12, 9, 256, 1, 8),
    (27, "int32_t", 14, 10, 256, 1, 8),
    (28, "int32_t", 13, 10, 256, 1, 8),
]


def main():
    cfg_h = os.path.join(CSRC, "hkt_cfg.h")
    s = open(cfg_h).read()
    rows = " \\\n".join(f"    X({c[0]}, {c[1]}, {c[2]}, {c[3]}, {c[4]}, {c[5]}, {c[6]})" for c in CFGS)
    s = re.sub(r"#define TSPGPU_TILED_CFGS\(X\) \\\n(?:    X\([^)]*\)(?: \\)?\n)+", f"#define TSPGPU_TILED_CFGS(X) \\\n{rows}\n", s)
    open(cfg_h, "w").write(s)
    for f in glob.glob(os.path.join(CSRC, "hkt_c*.hip")):
        os.remove(f)
    for c in CFGS:
        with open(os.path.join(CSRC, f"hkt_c{c[0]}.hip"), "w") as fh:
            fh.write(f"// K1 variant 5 instantiation {c[0]} (table: hkt_cfg.h)\n#include \"hk_tiled.h\"\nnamespace tspgpu {{\n"
                     f"template hipError_t launch_tiled_n<{c[1]}, {c[2]}, {c[3]}, {c[4]}, {c[5]}, {c[6]}>(const TiledArgs &);\n"
                     f"}}  // namespace tspgpu\n")


if __name__ == "__main__":
    main()
