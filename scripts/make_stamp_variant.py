"""Write an instrumented copy of vq_kernels.hip with s_memtime stamps in the
filter kernel's row loop (wave 0 of workgroups 0..255, first 16 iterations)
and an exported reader, vqgnn_dbg_vq_times; build it as a variant library:
  python scripts/make_stamp_variant.py /tmp/vq_time.hip
  bash scripts/build_variant.sh vqtime vq_kernels.hip /tmp/vq_time.hip
then VQGNN_LIB=vq-gnn_amd/lib/ab_vqtime.so python scripts/assign_phase_stamps.py
(measurement only: the product library has no stamps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(ROOT, "vq-gnn_amd", "csrc", "vq_kernels.hip")).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:60]
    s = s.replace(old, new)


rep("constexpr int kFltSlack = 32;", "__device__ unsigned long long g_vq_times[256 * 16 * 8];\n"
    "constexpr int kFltSlack = 32;")
loop = "for (int it = 0; it < n_iters; ++it) {"
second = s.index(loop, s.index(loop) + 10)          # the filter kernel's row loop
s = (s[:second] + loop + "\n    const bool dbg = blockIdx.x < 256 && wave == 0 && it < 16;\n"
     "    const unsigned long long t0 = __builtin_amdgcn_s_memtime();\n"
     "    unsigned long long t1 = 0, t2 = 0, t3 = 0;" + s[second + len(loop):])
rep("    bool ntie = !(sx < 65536.f);\n", "    bool ntie = !(sx < 65536.f);\n"
    "    t1 = __builtin_amdgcn_s_memtime();\n")
rep("      uint32_t kk[4];\n", "      t2 = __builtin_amdgcn_s_memtime();\n      uint32_t kk[4];\n")
rep("      if (dm < best) {                                // earlier chunk wins ties",
    "      t3 = __builtin_amdgcn_s_memtime();\n"
    "      if (dm < best) {                                // earlier chunk wins ties")
rep("""      }
    }
  }
  }   // pass""", """      }
    }
    if (dbg) {
      const unsigned long long t4 = __builtin_amdgcn_s_memtime();
      if (lane < 5) {
        const unsigned long long tv = lane == 0 ? t0 : lane == 1 ? t1 : lane == 2 ? t2
                                    : lane == 3 ? t3 : t4;
        g_vq_times[((size_t)blockIdx.x * 16 + it) * 8 + lane] = tv;
      }
    }
  }
  }   // pass""")
s += """
extern "C" int vqgnn_dbg_vq_times(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vqgnn::g_vq_times), (size_t)n * 8);
}
"""
open(sys.argv[1], "w").write(s)
