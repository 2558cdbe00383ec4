"""Bound the verdict's two-launch straggler deferral for exact mode by measurement
instead of building its state hand-off: diagnostic libraries whose adaptive loop stops after CAP RK45
attempts per env and skips the ground-event root (brentq), i.e. pass 1 of the two-launch design
without the spill of the deferred envs' loop state, and — launched on a small batch — a floor for
pass 2 (a 4-wave launch whose envs make at most CAP attempts).

    python tools/ab_exact_cap.py 2 1        # -> tools/ab/lib_cap2.so, tools/ab/lib_cap1.so

Outputs of these libraries are wrong by construction (timing only); the patch is applied to the
in-tree rocket_dopri5.inc for the build and reverted afterwards, so no diagnostic branch lives in
the product source.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
INC = os.path.join(ROOT, "rl_rocket_amd", "csrc", "rocket_dopri5.inc")

# (anchor, replacement): a per-env attempt counter, the cap at the top of each attempt, and the
# event lanes leaving before their dense output / brentq
PATCH = [
    ("    double g = y[EV], h_ev = 0.0;\n    for (;;) {\n",
     "    double g = y[EV], h_ev = 0.0;\n    int n_att = 0;\n    for (;;) {\n"),
    ("                if (!(h_abs >= min_step)) return -1;\n",
     "                if (!(h_abs >= min_step)) return -1;\n                if (n_att++ >= RR_EXACT_CAP) return 0;\n"),
    ("            if ((g <= 0 && g_new >= 0) || (g >= 0 && g_new <= 0)) {\n                if constexpr (!LEAN) return event_out();\n",
     "            if ((g <= 0 && g_new >= 0) || (g >= 0 && g_new <= 0)) {\n                return 1;\n"),
]


def main():
    from rl_rocket_amd.build import build_lib

    caps = [int(x) for x in sys.argv[1:]] or [2, 1]
    with open(INC) as f:
        orig = f.read()
    src = orig
    for a, b in PATCH:
        if src.count(a) != 1:
            raise SystemExit("anchor not found once: %r" % a[:60])
        src = src.replace(a, b)
    os.makedirs(os.path.join(ROOT, "tools", "ab"), exist_ok=True)
    try:
        with open(INC, "w") as f:
            f.write(src)
        for cap in caps:
            build_lib(os.path.join(ROOT, "tools", "ab", "lib_cap%d.so" % cap), defines=["RR_EXACT_CAP=%d" % cap])
    finally:
        with open(INC, "w") as f:
            f.write(orig)


if __name__ == "__main__":
    main()
