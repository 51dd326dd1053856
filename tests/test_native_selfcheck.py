"""CPU-only: the device H3 code (mosaic_amd/csrc/h3_device.h) compiled for the host must match the
oracle bit for bit -- h3_exact everywhere (glibc_math.h's restatement of libm against the oracle's
real glibc; validates the restatement and the x87 long-double emulation), h3_fast wherever it does not flag the point as ambiguous (validates the
projective fast path, the face lookup table, the table sine/cosine and the margin bounds).
Includes adversarial points built within 1e-9 hex units of cell edges, vertices and face centres."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_device_h3_code_on_host(tmp_path, oracle_lib):
    exe = tmp_path / "h3sc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "h3_host_selfcheck.cpp"),
                    os.path.join(ROOT, "oracle", "liboracle.so"), f"-Wl,-rpath,{os.path.join(ROOT, 'oracle')}"],
                   check=True)
    out = subprocess.run([str(exe), "400000", "11"], check=True, capture_output=True, text=True).stdout.split()
    bad_exact, bad_fast, ambiguous = map(int, out)
    assert bad_exact == 0 and bad_fast == 0
    assert ambiguous > 1000  # the adversarial quarter does exercise the exact path


def test_glibc_math_restatement_is_bit_exact(tmp_path):
    """mosaic_amd/csrc/glibc_math.h (the exact path's sincos / tan / acos / atan2 on the device)
    compiled for the host equals this image's glibc 2.35 libm bit for bit on 2e6 arguments per
    function: H3's argument ranges, thresholds between glibc's branches, huge arguments
    (__branred), zeros, infinities, NaN and random bit patterns."""
    exe = tmp_path / "gmsc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "glibc_math_selfcheck.cpp"), "-lm"], check=True)
    res = subprocess.run([str(exe), "2000000", "3"], capture_output=True, text=True)
    rows = [line.split() for line in res.stdout.split("\n") if line.strip()]
    assert {r[0] for r in rows} == {"sin", "cos", "tan", "acos", "atan2", "atan", "asin"}
    for name, n, bad in rows:
        assert int(n) > 1000000 and int(bad) == 0, (name, n, bad, res.stderr)
    assert res.returncode == 0


def test_h3_digit_pairs_equal_single_levels(tmp_path):
    """h3_device.h face_axial_to_h3 takes _faceIjkToH3's aperture-7 levels two at a time (the two
    centre maps compose to 7 x identity, so the digit pair depends only on the axial coordinates
    mod 7: kAxialPairs); it must equal the one-level form on every face and resolution."""
    exe = tmp_path / "pairs"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-I",
                    os.path.join(ROOT, "mosaic_amd", "csrc"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "h3_pairs_check.cpp")], check=True)
    n, bad = map(int, subprocess.run([str(exe), "2000000"], check=True, capture_output=True, text=True).stdout.split())
    assert n > 6_000_000 and bad == 0
