"""Kernel experiments: build variants of kernels_http.hip (text substitutions
applied to a copy) into tools/_exp/lib_<name>.so, linked with the library's
other objects.  Run on the GPU box with tools/exp_http.sh; each variant is
timed by tools/prof_http.py through CILIUM_AMD_LIB.  Variants are measuring
devices only (e.g. "no LDS read") — their verdicts are meaningless.

    python tools/exp_http.py build
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from cilium_amd import build as B  # noqa: E402

OUT = ROOT / "tools" / "_exp"
LDS_READ = ("  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + "
            "((st << 2) + (b << 2)));")
# keeps the walk's result live but never lets a meaningless state index the
# accept tables (variants that break the DFA must stay memory-safe)
C_STEP = ("""  uint32_t nx;
  asm("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:WORD_0 src1_sel:DWORD\\n\\t"
      "s_nop 1\\n\\t"
      "v_cndmask_b32_sdwa %0, %3, %1, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
      : "=v"(nx)
      : "v"(e), "v"(st), "v"(dflt)
      : "vcc");
  return nx;""", """  return (uint16_t)e == (uint16_t)st ? (e >> 16) : dflt;""")
K = "constexpr int kTilesPerWave = 1;"
DFLT = "  const uint32_t dflt = st >= self_lo ? st : 0u;\n  // nx = e.lo == st ? e.hi : dflt\n"
NODFA = ("  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cells) + ((st << 2) + (b << 2)));",
         "  const uint32_t e = (st * 33u + b) | 0x10000u;")
WALK = "    for (int i = 0; i < 16; ++i) st = comb_step(blk, self_lo, st, get_byte(unit[k], i));"
STAGE = "        for (uint32_t i = threadIdx.x; i < pg.cell_count; i += blockDim.x) lcells[i] = T.cells[pg.cell_begin + i];"
NOWALK = (WALK, "    for (int i = 0; i < 1; ++i) st ^= unit[k].x ^ unit[k].y ^ unit[k].z ^ unit[k].w;")
ATOM = ("    if (real && s_cnt[0]) atomicAdd(", "    if (real && s_cnt[0] == 0xFFFFFFFFu) atomicAdd(")
ATOM2 = ("    if (real && s_cnt[1]) atomicAdd(", "    if (real && s_cnt[1] == 0xFFFFFFFFu) atomicAdd(")
NOREMOTE = [("  unsigned long long k0 = T.rhash_keys[rh];\n  uint32_t v0 = T.rhash_vals[rh];",
             "  unsigned long long k0 = rkey;\n  uint32_t v0 = pg.default_remote;"),
            ("      r0 = T.masks[row];\n      r1 = T.masks[row + 1];\n      __builtin",
             "      r0 = row;\n      r1 = row;\n      __builtin")]
VARIANTS = {
    "base": [],
    "nowalk": [NODFA, NOWALK],
    "pftt": [("""      for (uint32_t t = ch.first_tile + wave; t < tend; t += nw) {
        const HttpTile tt = ttab[t];
        const TileRef tb = tile_ref(tiles, tt);""", """      HttpTile nxt = ttab[min(ch.first_tile + wave, tend - 1)];
      for (uint32_t t = ch.first_tile + wave; t < tend; t += nw) {
        const HttpTile tt = nxt;
        nxt = ttab[min(t + nw, tend - 1)];  // next tile's entry loads under this tile's walk
        const TileRef tb = tile_ref(tiles, tt);""")],
    "deal2": [("constexpr uint32_t kDealRun = 4;", "constexpr uint32_t kDealRun = 2;")],
    "deal8": [("constexpr uint32_t kDealRun = 4;", "constexpr uint32_t kDealRun = 8;")],
    "deal16": [("constexpr uint32_t kDealRun = 4;", "constexpr uint32_t kDealRun = 16;")],
}


def build_variant(name, subs):
    src = (B.CSRC / "kernels_http.hip").read_text()
    for a, b in subs:
        assert a in src, (name, a)
        src = src.replace(a, b)
    OUT.mkdir(exist_ok=True)
    f = OUT / f"kernels_http_{name}.hip"
    f.write_text(src.replace('"../../include/cilium_gpu.h"', f'"{ROOT}/include/cilium_gpu.h"'))
    obj = OUT / f"kernels_http_{name}.o"
    cmd = [B.HIPCC, *B._flags("x.hip"), "-I", str(B.CSRC), "-c", str(f), "-o", str(obj)]
    subprocess.run(cmd, check=True)
    others = [B.BUILD / (s + ".o") for s in B.SOURCES if s != "kernels_http.hip"]
    lib = OUT / f"lib_{name}.so"
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *map(str, others), str(obj), "-o",
                    str(lib)], check=True)
    print("built", lib)


if __name__ == "__main__":
    B.build(verbose=False)
    names = sys.argv[2:] or list(VARIANTS)
    for n in names:
        build_variant(n, VARIANTS[n])
