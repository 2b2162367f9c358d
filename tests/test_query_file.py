"""The worker's query-file reader (csrc/cpd_io.cpp read_query_file: one
buffer, lines parsed by up to T threads) against the format
process_query.send_queries writes (process_query.py:93-96: "{n}\\n" then n
"s t" lines): every thread count gives the file's pairs in order; blank
lines are skipped; a bad line, a count that disagrees with the lines and a
missing header are errors.  Host only: the harness is compiled from the
library's sources with g++."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-oracle-search_amd", "csrc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("qf") / "qf")
    subprocess.run([gxx, "-O2", "-std=c++17", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
                    os.path.join(CSRC, "cpd_io.cpp"), os.path.join(ROOT, "tests", "query_file_check.cpp"),
                    "-o", out, "-lpthread"], check=True, capture_output=True, timeout=240)
    return out


def _read(harness, path, threads):
    p = subprocess.run([harness, path, str(threads)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout


def test_pairs_in_order_any_thread_count(harness, tmp_path):
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 250_000):
        s = rng.integers(0, 2**32 - 1, n, dtype=np.uint64)
        t = rng.integers(0, 4_000_000, n, dtype=np.uint64)
        path = str(tmp_path / f"q{n}")
        body = "".join(f"{a} {b}\n" for a, b in zip(s.tolist(), t.tolist()))
        if n == 7:  # blank lines and CRLF endings are tolerated
            body = body.replace("\n", "\r\n", 2) + "\n\n"
        with open(path, "w") as f:
            f.write(f"{n}\n" + body)
        want = f"{n}\n" + "".join(f"{a} {b}\n" for a, b in zip(s.tolist(), t.tolist()))
        for threads in (1, 3, 16):
            assert _read(harness, path, threads) == want, (n, threads)


def test_errors(harness, tmp_path):
    cases = {"bad_line": "3\n1 2\n3 x\n5 6\n", "count": "4\n1 2\n3 4\n",
             "no_header": "\n1 2\n", "negative": "1\n-1 2\n"}
    for name, text in cases.items():
        path = str(tmp_path / name)
        with open(path, "w") as f:
            f.write(text)
        for threads in (1, 8):
            assert _read(harness, path, threads).startswith("ERR"), (name, threads)
    empty = str(tmp_path / "empty")
    open(empty, "w").close()
    assert _read(harness, empty, 4) == "0\n"
