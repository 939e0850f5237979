"""The count kernels' word-parallel k-mer windows (csrc/ks_kmer_swar.h)
against the byte-serial walk they replaced (N-free runs, sequence starts,
quirk Q1 of kmer_spans.c:142-144), on the host: tests/swar_check.cpp over
random 32-byte lane windows, every k in [1, 15].  The GPU count tests
(test_gpu_configs.py, test_ingest.py) then compare the counts with the
oracle."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_swar_windows_equal_the_byte_walk(tmp_path):
    exe = str(tmp_path / "swar_check")
    for flags in (["-O2"], ["-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]):
        r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wno-unknown-pragmas", *flags, "-o", exe,
                            os.path.join(HERE, "swar_check.cpp")], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        r = subprocess.run([exe, "100000"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.startswith("ok "), r.stdout
