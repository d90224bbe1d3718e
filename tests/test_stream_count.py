"""The online stream's bounded frame count (csrc/online.h stream_next_count),
compiled from the header and run on the host (CPU only): past 2^30 it drops by a
multiple of 2W, keeping the ring slot, the launch parity (the online kernel's
activation tag) and a count far above the window's left-edge clamp."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SRC = r'''
#include <cstdio>
#include "online.h"
int main() {
    const int Ws[] = {3, 9, 21, 65, 129, 4097};
    for (int W : Ws) {
        // every step: +1, or the wrap; the wrap keeps c mod 2W and stays >= 2^29
        long long seen_wrap = 0;
        int c = (1 << 30) - 3 * W;
        long long ref = c;   // the unbounded count
        for (int i = 0; i < 6 * W + 10; ++i) {
            const int n = tik::stream_next_count(c, W);
            ++ref;
            if (n < 0 || n >= (1 << 30)) { printf("range %d %d\n", W, n); return 1; }
            if ((ref - n) % (2LL * W) != 0) { printf("residue %d\n", W); return 1; }
            if (n != c + 1) { ++seen_wrap; if (n < (1 << 29)) { printf("low %d %d\n", W, n); return 1; } }
            c = n;
        }
        if (seen_wrap != 1) { printf("wraps %d %lld\n", W, seen_wrap); return 1; }
        // small counts: plain increments
        for (int x = 0; x < 1000; ++x) if (tik::stream_next_count(x, W) != x + 1) { printf("inc %d\n", x); return 1; }
    }
    printf("ok\n");
    return 0;
}
'''


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_stream_next_count(tmp_path):
    src = tmp_path / "count.hip"
    src.write_text(SRC)
    exe = tmp_path / "count"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17",
                        f"-I{os.path.join(REPO, 'temporal_inverse_kinematics_amd', 'csrc')}", str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
