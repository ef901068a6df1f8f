"""Generates mb_bank.hip: SIMD cycles per wave64 VOP3 integer instruction by VGPR operand banks.

Question (round 3): the VOP3 ops of the SHA-1/CRC kernels (v_add3, v_bitop3, v_alignbit) measured
at ~4 SIMD cycles each at 2-4 waves per SIMD (mb_rate), against the guide's 2 cycles for v_fma_f32
-- but mb_rate's ops read one register twice (`%0, %1, %1`).  Is the 4 a property of the opcode or
of the operands (same register / same VGPR bank, bank = register index mod 4)?  Every timed loop is
one asm block over explicit registers (sources v32..v47 never written in the loop, destinations
v48..v95), so the register allocation is exactly what the name says.  Not part of the product.

    python tools/microbench/gen_mb_bank.py [2] && hipcc --offload-arch=gfx950 -O3 \
        -o tools/microbench/mb_bank tools/microbench/mb_bank.hip && tools/microbench/mb_bank
"""
import os

N_PER_ITER = 64  # instructions per loop iteration


def src(bank, k):
    """k-th source register of VGPR bank `bank` (v32..v47: four per bank)."""
    return f"v{32 + 4 * (k % 4) + bank}"


def dst(i, bank=None):
    if bank is None:
        return f"v{48 + (i % 48)}"
    return f"v{48 + 4 * (i % 12) + bank}"


def variants():
    v = {}
    v["add3 banks 1,2,3"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["add3 banks 1,1,1"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, {src(1, i + 2)}"
    v["add3 banks 1,1,2"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, {src(2, i)}"
    v["add3 reg x,x,y"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(1, i)}, {src(2, i)}"
    v["add3 banks 1,2,3 dst bank 1"] = lambda i: f"v_add3_u32 {dst(i, 1)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["add3 banks 1,2,3 dst bank 0"] = lambda i: f"v_add3_u32 {dst(i, 0)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["add3 banks 1,2 + sgpr"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, s40, {src(2, i)}"
    v["add3 banks 1,2 + const"] = lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, 7, {src(2, i)}"
    v["bitop3 banks 1,2,3"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)} bitop3:0x96"
    v["bitop3 banks 1,1,1"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, {src(1, i + 2)} bitop3:0x96"
    v["alignbit rot x,x"] = lambda i: f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(1, i)}, 27"
    v["alignbit banks 1,2"] = lambda i: f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, 27"
    v["alignbit banks 1,1"] = lambda i: f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, 27"
    v["fma_f32 banks 1,2,3"] = lambda i: f"v_fma_f32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["fma_f32 reg x,y,y"] = lambda i: f"v_fma_f32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(2, i)}"
    v["add_u32_e32 banks 1,2"] = lambda i: f"v_add_u32_e32 {dst(i)}, {src(1, i)}, {src(2, i)}"
    v["add_u32_e32 banks 1,1"] = lambda i: f"v_add_u32_e32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}"
    v["add_u32_e64 banks 1,2"] = lambda i: f"v_add_u32_e64 {dst(i)}, {src(1, i)}, {src(2, i)}"
    v["lshlrev sdwa byte1"] = lambda i: (f"v_lshlrev_b32_sdwa {dst(i)}, {src(1, i)}, {src(2, i)} dst_sel:DWORD "
                                         "dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
    v["perm banks 1,2 + sgpr"] = lambda i: f"v_perm_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, s41"
    return v


def variants2():
    """Second pass: partial bank conflicts, and full-rate candidates for rotates / byte indices."""
    v = {}
    v["bitop3 banks 1,1,2"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, {src(2, i)} bitop3:0x96"
    v["bitop3 banks 1,2,1"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(1, i + 1)} bitop3:0x96"
    v["bitop3 reg x,x,y"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(1, i)}, {src(2, i)} bitop3:0x96"
    v["bitop3 banks 1,2 + sgpr"] = lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, s40 bitop3:0x96"
    v["bitop3 banks 1,2,3 dst bank 1"] = lambda i: f"v_bitop3_b32 {dst(i, 1)}, {src(1, i)}, {src(2, i)}, {src(3, i)} bitop3:0x96"
    v["bfe_u32 bank 1"] = lambda i: f"v_bfe_u32 {dst(i)}, {src(1, i)}, 14, 10"
    v["lshrrev_b32_e32"] = lambda i: f"v_lshrrev_b32_e32 {dst(i)}, 22, {src(1, i)}"
    v["and_b32_e32 const"] = lambda i: f"v_and_b32_e32 {dst(i)}, 0x3fc, {src(1, i)}"
    v["lshl_or_b32 banks 1,2"] = lambda i: f"v_lshl_or_b32 {dst(i)}, {src(1, i)}, 5, {src(2, i)}"
    v["lshl_add_u32 banks 1,2"] = lambda i: f"v_lshl_add_u32 {dst(i)}, {src(1, i)}, 5, {src(2, i)}"
    v["xad_u32 banks 1,2,3"] = lambda i: f"v_xad_u32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["and_or_b32 banks 1,2,3"] = lambda i: f"v_and_or_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["or3_b32 banks 1,2,3"] = lambda i: f"v_or3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["bfi_b32 banks 1,2,3"] = lambda i: f"v_bfi_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"
    v["alignbyte banks 1,2"] = lambda i: f"v_alignbyte_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, 1"
    v["xor_b32_e64 banks 1,2"] = lambda i: f"v_xor_b32_e64 {dst(i)}, {src(1, i)}, {src(2, i)}"
    v["mul_u32_u24 banks 1,2"] = lambda i: f"v_mul_u32_u24_e32 {dst(i)}, {src(1, i)}, {src(2, i)}"
    v["pk_add_u16 banks 1,2"] = lambda i: f"v_pk_add_u16 {dst(i)}, {src(1, i)}, {src(2, i)}"
    v["SHA mix, bitop3 1,2,3"] = lambda i: [f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(1, i)}, 27",
                                             f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)} bitop3:0x96",
                                             f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}",
                                             f"v_add_u32_e32 {dst(i)}, {src(1, i)}, {src(2, i)}"][i % 4]
    v["SHA mix, bitop3 1,1,2"] = lambda i: [f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(1, i)}, 27",
                                             f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(1, i + 1)}, {src(2, i)} bitop3:0x96",
                                             f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}",
                                             f"v_add_u32_e32 {dst(i)}, {src(1, i)}, {src(2, i)}"][i % 4]
    return v


HEAD = r'''// GENERATED by gen_mb_bank.py -- see its docstring.  Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;}}while(0)
typedef void (*kfn)(uint32_t*, uint64_t*, int);
struct K { const char* name; kfn f; const char* exec; };
'''


def kernel(idx, fn, exec_mode):
    body = "\n".join(f'    "{fn(i)}\\n"' for i in range(N_PER_ITER))
    clob = ", ".join(f'"v{r}"' for r in range(32, 96))
    init = "\n".join(f'    "v_add_u32_e32 v{r}, {r}, %[x]\\n"' for r in range(32, 48))
    exec_set = {"full": "", "lo32": '    "s_mov_b32 exec_hi, 0\\n"', "one": '    "s_mov_b64 exec, 1\\n"'}[exec_mode]
    return f'''
__global__ __launch_bounds__(1024) void k{idx}_{exec_mode}(uint32_t* out, uint64_t* cyc, int iters) {{
  uint32_t x = threadIdx.x * 2654435761u;
  int n = iters;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(
    "s_mov_b64 s[42:43], exec\\n"
    "s_mov_b32 s40, 0x9E3779B9\\n"
    "s_mov_b32 s41, 0x00010203\\n"
{init}
{exec_set}
    "1:\\n"
{body}
    "s_sub_u32 %[n], %[n], 1\\n"
    "s_cmp_lg_u32 %[n], 0\\n"
    "s_cbranch_scc1 1b\\n"
    "s_mov_b64 exec, s[42:43]\\n"
    "v_xor_b32_e32 %[x], v48, %[x]\\n"
    : [n] "+s"(n), [x] "+v"(x)
    :
    : {clob}, "s40", "s41", "s42", "s43", "scc");
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}}
'''


MAIN = r'''
int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int iters = 20000;
  uint32_t* out; uint64_t* cyc;
  CK(hipMalloc(&out, sizeof(uint32_t) * cus * 64 * 4 * 4));
  CK(hipMalloc(&cyc, sizeof(uint64_t) * cus * 4 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  printf("%d CUs; %d instructions per wave; SIMD cycles per wave64 instruction (s_memtime of the slowest wave)\n",
         cus, iters * NPI);
  for (const K& k : ks) {
    for (int w : {1, 2, 4}) {
      const int threads = 64 * 4 * w;
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, 10);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(threads), 0, 0, out, cyc, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<uint64_t> c(cus * 4 * w);
      CK(hipMemcpy(c.data(), cyc, c.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      uint64_t mx = 0; for (auto v : c) mx = v > mx ? v : mx;
      const double per_simd = double(w) * iters * NPI;
      printf("%-30s exec=%-4s waves/SIMD=%d  %8.3f ms  SIMD cyc/instr %.2f (memtime) %.2f (wall @2.4GHz)  clk %.2f GHz\n",
             k.name, k.exec, w, ms, double(mx) / per_simd, ms * 1e-3 * 2.4e9 / per_simd, double(mx) / (ms * 1e6));
    }
  }
  return 0;
}
'''


def variants3():
    """Third pass: streams mixing half-rate (H: alignbit / add3) and full-rate (F: bitop3 with
    three banks, VOP2 add) instructions in fixed patterns."""
    H = {"A": lambda i: f"v_alignbit_b32 {dst(i)}, {src(1, i)}, {src(1, i)}, 27",
         "3": lambda i: f"v_add3_u32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)}"}
    F = {"B": lambda i: f"v_bitop3_b32 {dst(i)}, {src(1, i)}, {src(2, i)}, {src(3, i)} bitop3:0x96",
         "a": lambda i: f"v_add_u32_e32 {dst(i)}, {src(1, i)}, {src(2, i)}",
         "x": lambda i: f"v_xor_b32_e32 {dst(i)}, {src(2, i)}, {src(3, i)}"}
    ops = {**H, **F}
    v = {}
    for pat in ["Ba", "Bx", "aBxB", "AB", "Aa", "3B", "3a", "ABBB", "AaBx", "AAB", "AABa", "A3Ba", "AAAB", "A3", "AA3Ba"]:
        v["mix " + pat] = (lambda pat: lambda i: ops[pat[i % len(pat)]](i))(pat)
    return v


def main():
    import sys
    second = len(sys.argv) > 1 and sys.argv[1] == "2"
    third = len(sys.argv) > 1 and sys.argv[1] == "3"
    out = [HEAD, f"#define NPI {N_PER_ITER}\n"]
    table = []
    for idx, (name, fn) in enumerate((variants3() if third else variants2() if second else variants()).items()):
        modes = ["full"]
        if name in ("add3 banks 1,2,3", "alignbit rot x,x", "add_u32_e32 banks 1,2"):
            modes += ["lo32", "one"]
        for m in modes:
            out.append(kernel(idx, fn, m))
            table.append(f'  {{"{name}", k{idx}_{m}, "{m}"}},')
    out.append("K ks[] = {\n" + "\n".join(table) + "\n};\n")
    out.append(MAIN)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mb_bank3.hip" if third else "mb_bank2.hip" if second else "mb_bank.hip")
    with open(path, "w") as f:
        f.write("".join(out))


if __name__ == "__main__":
    main()
