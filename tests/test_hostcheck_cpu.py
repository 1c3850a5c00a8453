"""Sanitizer build of the host-side code: the per-lane device
logic of csrc/gz_bitboard.h compiled for the host (tests/hosttest/gz_hosttest.cpp)
and the C oracle (oracle/gz_oracle.c), both with -fsanitize=address,undefined,
driven by tests/hosttest/gz_hostcheck.cpp: the bitboard rollout policy and whole
rollouts equal the oracle's on random positions, and the oracle's MCTS search and
self-play game run clean.  (GPU sanitizers are not available on the pool.)"""
import os
import shutil
import subprocess

import pytest

from conftest import REPO


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc / g++")
def test_bitboard_and_oracle_under_asan_ubsan(tmp_path):
    ht = os.path.join(REPO, "tests", "hosttest")
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    oracle_o = str(tmp_path / "gz_oracle.o")
    subprocess.run(["gcc", "-std=c11", "-ffp-contract=off", *san, "-c", os.path.join(REPO, "oracle", "gz_oracle.c"),
                    "-o", oracle_o], check=True)
    exe = str(tmp_path / "gz_hostcheck")
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", *san, os.path.join(ht, "gz_hostcheck.cpp"),
                    os.path.join(ht, "gz_hosttest.cpp"), oracle_o, "-lm", "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "600"], capture_output=True, text=True, env=env, timeout=600)
    print(r.stdout[-2000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "0 mismatches" in r.stdout
