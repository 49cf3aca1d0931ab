"""Sanitizer runs on the CPU ("race detection / sanitizers"): the host harnesses
of tests/native -- which compile every engine header (the packed 8-B / 16-B record indexing of
search_core.h, the register rollouts, CAP, the rs-doko sampler, the AlphaZero core, the IMPI
sampler, the Dirichlet draws) together with the oracle restatement -- built with
-fsanitize=address,undefined -fno-sanitize-recover=all (`make asan`), on reduced inputs; and the
oracle's own KAT / golden-trace tests against the sanitized oracle library loaded into a Python
process with the sanitizer runtimes preloaded.  Any finding aborts the run and fails the test.
GPU code is not sanitized here (GPU AddressSanitizer is not available on this pool)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
ORACLE = os.path.join(ROOT, "oracle")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def asan_bins():
    subprocess.run(["make", "-s", "-j8", "-C", NATIVE, "asan"], check=True)
    return os.path.join(NATIVE, "asan")


# (binary, arguments, minimum of the count the harness prints after "OK")
CASES = [
    ("search_check", (3, 300, 5), 3),            # 16-B records
    ("search_check8", (3, 400, 9), 3),           # 8-B packed records, pair loads, resolved chain heads
    ("search_check8", (2, 1000, 11, 2), 2),      # 8-B records at the C3 iteration count
    ("search_check16l", (1, 4200, 21), 1),       # 16-B long records past the 24-bit cross products
    ("search_check32", (3, 300, 5), 3),          # 32-B records (cached means)
    ("uct_pick_check8", (100000, 4), 100000),    # the filtered pick over 8-B record blocks
    ("cap_check", (30, 3), 1000),
    ("fdo_engine_check", (40, 11), 1000),
    ("do_engine_check", (30, 7), 1000),
    ("az_check", (20, 100, 5), 120),
    ("dirichlet_check", (2000, 3), 376000),
    ("libm_check", (65537, 8), 65536),
    ("assign_check", (30, 3), 1000),
    ("ar_check", (30, 3, 9), 200),
]


@pytest.mark.parametrize("binary,args,least", CASES, ids=["%s-%s" % (c[0], "-".join(map(str, c[1]))) for c in CASES])
def test_harness_under_asan_ubsan(asan_bins, binary, args, least):
    out = subprocess.run([os.path.join(asan_bins, binary)] + [str(a) for a in args], capture_output=True, text=True,
                         timeout=300, env=ENV)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-4000:]
    assert out.stdout.startswith("OK"), out.stdout
    assert int(out.stdout.split()[1]) >= least


def test_oracle_library_under_asan_ubsan():
    """The oracle's rule KATs and golden traces with the sanitized liboracle_doko.so."""
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    lib = os.path.join(ORACLE, "_asan", "liboracle_doko.so")
    rt = [subprocess.run(["gcc", "-print-file-name=" + n], capture_output=True, text=True, check=True).stdout.strip()
          for n in ("libasan.so", "libubsan.so")]
    assert all(os.path.isabs(p) and os.path.exists(p) for p in rt), rt
    env = dict(ENV, LD_PRELOAD=":".join(rt), ORACLE_LIB=lib)
    probe = ("import sys; sys.path.insert(0, %r); import oracle_lib as ol; ol.lib(); "
             "m = open('/proc/self/maps').read(); assert %r in m and 'libasan' in m, 'sanitized oracle not loaded'; "
             "print('loaded')") % (os.path.join(ROOT, "tests"), lib)
    out = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0 and "loaded" in out.stdout, out.stdout + out.stderr
    out = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                          os.path.join(ROOT, "tests", "test_rule_kats.py"),
                          os.path.join(ROOT, "tests", "test_oracle_golden.py")],
                         capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-4000:]
