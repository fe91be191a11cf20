"""CPU: the counted-wait guard.  The GEMM kernels' s_waitcnt vmcnt
immediates are derived from constexpr op counts (csrc/common.hpp vm_wait / vm_wait_stages), and the
MICLIP_VMCHECK build -- which `make` compiles beside the product objects -- counts the VMEM ops a
code section issues and calls an undefined function when the count differs from the one its wait was
derived from, so the device link fails.  Checked here on a small kernel written the same way (hipcc
cross-compiles for gfx950 without a GPU): a matching count links, a count one short fails with the
guard's symbol named; and the product build's counting objects exist."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG

CSRC = os.path.join(PKG, "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

KERNEL = r'''
#include "common.hpp"
// an "epilogue" of BLOCKS blocks of STORES stores each, and the wait derived from that count
template <int BLOCKS, int STORES, int CLAIMED>
__global__ void k(float* o) {
  int vm = 0;
#pragma unroll
  for (int b = 0; b < BLOCKS; ++b)
#pragma unroll
    for (int s = 0; s < STORES; ++s) {
      o[(b * STORES + s) * 64 + threadIdx.x] = (float)b;
      if (MICLIP_VMCHECK) ++vm;
    }
  if (MICLIP_VMCHECK) vm_count_check<CLAIMED>(vm);
  vm_wait<CLAIMED < VM_MAX ? CLAIMED : VM_MAX>();
}
template __global__ void k<8, 2, CLAIM>(float*);
'''


def _compile(tmp_path, claim):
    src = tmp_path / f"vm_{claim}.hip"
    src.write_text(KERNEL)
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{CSRC}", "-DMICLIP_VMCHECK=1",
                        f"-DCLAIM={claim}", "--offload-device-only", "-x", "hip", "-c", str(src),
                        "-o", str(tmp_path / f"vm_{claim}.o")], capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_vm_count_guard_links_only_on_a_matching_count(tmp_path):
    rc, log = _compile(tmp_path, 16)          # 8 blocks x 2 stores: the count the code issues
    assert rc == 0, log
    rc, log = _compile(tmp_path, 15)          # a hand count one short: the round-5 bug's shape
    assert rc != 0 and "miclip_vmcnt_count_mismatch" in log, log


def test_counting_objects_are_part_of_the_build():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    assert "VMCHECK_SRCS = gemm.hip gemm_8q.hip gemm_mx.hip" in mk
    assert "$(OUT): $(OBJS) $(VMCHECK)" in mk and "$(AB_OUT): $(AB_OBJS) $(AB_VMCHECK)" in mk
    if shutil.which("make") and os.path.exists(os.path.join(CSRC, "build")):
        for f in ("gemm.hip.o", "gemm_8q.hip.o", "gemm_mx.hip.o"):
            assert os.path.exists(os.path.join(CSRC, "build", "vmcheck", f)), f
