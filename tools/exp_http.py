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
# Substitutions on the current kernels_http.hip.  Variants are measuring
# devices; "nowalk" breaks the verdicts on purpose (memory-safe: the walk
# result stays live but never indexes the accept tables).
WALK_N = """#pragma unroll
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int i = 0; i < 16; ++i) st = comb_step(blk, self_lo, st, get_byte(unit[k], i));
  }"""
NOWALK = (WALK_N, """#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" ::"v"(unit[k].x), "v"(unit[k].y), "v"(unit[k].z), "v"(unit[k].w));""")
EARLY = (WALK_N, """#pragma unroll
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int i = 0; i < 16; ++i) st = comb_step(blk, self_lo, st, get_byte(unit[k], i));
    if (k + 1 < N && !__any(st != 0)) break;
  }""")
NOCTR = ("""  count_hits(T, pg, hit, s_hits, lane);
  out[(size_t)t * kWave + lane] = (uint8_t)verdict;""", """  out[(size_t)t * kWave + lane] = (uint8_t)verdict;""")
VARIANTS = {
    "base": [],
    "nosort": [("http_pack.cc", "  if (build) {\n    // each bucket sorted as", "  if (false) {\n    // each bucket sorted as")],
    "lensort": [("http_pack.cc", "        if (a.pre[0] != b.pre[0]) return a.pre[0] < b.pre[0];",
                 "        if (a.len != b.len) return a.len < b.len;\n        if (a.pre[0] != b.pre[0]) return a.pre[0] < b.pre[0];")],
}
# Kafka wire decode variants (kernels_kafka.hip): thread count / LDS stage.
def _kw(threads, stage):
    return [("kernels_kafka.hip", "constexpr uint32_t kKwThreads = 256;", f"constexpr uint32_t kKwThreads = {threads};"),
            ("kernels_kafka.hip", "constexpr uint32_t kKwStage = 4096;", f"constexpr uint32_t kKwStage = {stage};")]


VARIANTS.update({
    "kw_base": [],
    "kw_t256_s4k": _kw(256, 4096),
    "kw_t256_s2k": _kw(256, 2048),
    "kw_nostage": _kw(256, 0),
    "kw_nostage_t128": _kw(128, 0),
    "kw_nocrc": [("kernels_kafka.hip", "    uint32_t c = 0xFFFFFFFFu;\n    uint32_t h = (4u",
                  "    if (n > 0) return p[0];\n    uint32_t c = 0xFFFFFFFFu;\n    uint32_t h = (4u")],
})


# L4 (kernels.hip): tuples per lane per iteration; counters skipped (a
# measuring device: the per-entry counters stay zero).
def _l4t(k):
    return [("kernels.hip", "constexpr uint32_t kL4Tuples = 4;", f"constexpr uint32_t kL4Tuples = {k};")]


_NOPIPE = ("kernels.hip", "constexpr bool kL4Pipe = true;", "constexpr bool kL4Pipe = false;")
VARIANTS.update({
    "l4_pipe4": _l4t(4),
    "l4_pipe8": _l4t(8),
    "l4_nopipe4": _l4t(4) + [_NOPIPE],
    "l4_nopipe8": _l4t(8) + [_NOPIPE],
    "l4_noctr": [("kernels.hip", "      if (which) l4_count(t, lcnt, val & 0xFFFF, w[u][2]);", "")],
    # prefilter: addresses per lane (v4, v6)
    "lpm_4_2": [("kernels.hip", "constexpr uint32_t kLpmV4 = 4, kLpmV6 = 2;", "constexpr uint32_t kLpmV4 = 4, kLpmV6 = 2;")],
    "lpm_8_4": [("kernels.hip", "constexpr uint32_t kLpmV4 = 4, kLpmV6 = 2;", "constexpr uint32_t kLpmV4 = 8, kLpmV6 = 4;")],
    "lpm_4_4": [("kernels.hip", "constexpr uint32_t kLpmV4 = 4, kLpmV6 = 2;", "constexpr uint32_t kLpmV4 = 4, kLpmV6 = 4;")],
    # HTTP: dynamic (ticket) vs static chunk dealing
    "h_dyn": [],
    "h_static": [("constexpr bool kDynamicDeal = true;", "constexpr bool kDynamicDeal = false;")],
    # occupancy vs spills: 8 waves/SIMD caps VGPRs at 64 (40 B/lane of scratch)
    "h_w7": [("amdgpu_waves_per_eu(8, 8)", "amdgpu_waves_per_eu(7, 8)")],
    "h_w6": [("amdgpu_waves_per_eu(8, 8)", "amdgpu_waves_per_eu(6, 8)")],
    # next-tile prefetch depth and the rolling unit window
    "h_pre2": [("constexpr int kPre = 1;", "constexpr int kPre = 2;")],
    "h_win2": [("constexpr int kWin = N < 4 ? (N > 0 ? N : 1) : 4;", "constexpr int kWin = N < 2 ? (N > 0 ? N : 1) : 2;")],
    "h_win3": [("constexpr int kWin = N < 4 ? (N > 0 ? N : 1) : 4;", "constexpr int kWin = N < 3 ? (N > 0 ? N : 1) : 3;")],
    # nontemporal meta / prefetched-unit loads off (the in-walk unit loads stay nontemporal)
    "h_nt_units_only": [("#define NT_META(p) ld_nt(p)\n#define NT_PRE(p) ld_nt(p)", "#define NT_META(p) (*(p))\n#define NT_PRE(p) (*(p))")],
    "h_ntout": [("  out[(size_t)t * kWave + lane] = (uint8_t)verdict;\n  n_allow += counted && verdict;",
                 "  __builtin_nontemporal_store((uint8_t)verdict, out + (size_t)t * kWave + lane);\n  n_allow += counted && verdict;")],
    "h_old": [("#define NT_META(p) ld_nt(p)\n#define NT_PRE(p) ld_nt(p)", "#define NT_META(p) (*(p))\n#define NT_PRE(p) (*(p))"),
              ("unit[k] = k < kPre ? cur.u[k < kPre ? k : 0] : ld_nt(tr.units + k * kWave + lane);",
               "unit[k] = k < kPre ? cur.u[k < kPre ? k : 0] : tr.units[k * kWave + lane];"),
              ("unit[k % kWin] = ld_nt(tr.units + (k + kWin) * kWave + lane);",
               "unit[k % kWin] = tr.units[(k + kWin) * kWave + lane];")],
    "h_nt_nometa": [("#define NT_META(p) ld_nt(p)", "#define NT_META(p) (*(p))")],
    "h_win6": [("constexpr int kWin = N < 4 ? (N > 0 ? N : 1) : 4;", "constexpr int kWin = N < 6 ? (N > 0 ? N : 1) : 6;")],
})


# Raw HTTP path (kernels_http_raw.hip): LDS stage per wave, code maps in LDS
# (occupancy: the stage and the code maps set how many workgroups fit a CU).
def _rs(stage):
    return [("kernels_http_raw.hip", "constexpr uint32_t kStage = 6144;", f"constexpr uint32_t kStage = {stage};")]


_NOCODES = ("kernels_http_raw.hip", "return (size_t)R.nprogs * 256 <= 4 * 1024; }", "return false; }")
VARIANTS.update({
    "raw_base": [],
    "raw_s6k": _rs(6144),
    "raw_s4k": _rs(4096),
    "raw_nocodes": [_NOCODES],
    "raw_s6k_nocodes": _rs(6144) + [_NOCODES],
    "raw_s5k": _rs(5120),
    "raw_s5632": _rs(5632),
    "raw_s7k": _rs(7168),
    "raw_s5k_nocodes": _rs(5120) + [_NOCODES],
    "raw_s5632_nocodes": _rs(5632) + [_NOCODES],
    # measuring device (verdicts meaningless, memory-safe: separators and
    # zero padding only, all valid codes): emit without the strings
    "raw_ntstage": [("kernels_http_raw.hip", "      v = *reinterpret_cast<const uint4*>((uintptr_t)a);",
                     "      { typedef unsigned int v4u __attribute__((ext_vector_type(4))); const v4u x = "
                     "__builtin_nontemporal_load(reinterpret_cast<const v4u*>((uintptr_t)a)); v = make_uint4(x.x, x.y, x.z, x.w); }")],
    "raw_nostr": [("kernels_http_raw.hip", "      for (uint32_t k = 0; k < L; k += 4) {  // a quad",
                   "      for (uint32_t k = 0; k < 0; k += 4) {  // a quad")],
    # the scan's phases timed with the shader clock (printed by one wave)
    "raw_clocks": [("kernels_http_raw.hip", "#include <hip/hip_runtime.h>\n", "#include <hip/hip_runtime.h>\n#define CG_RAW_CLOCKS 1\n")],
    # raw_build_kernel measuring devices / variants: no class coding (verdicts
    # meaningless), nontemporal record loads, nontemporal tile stores
    "rb_nocode": [("kernels_http_raw.hip", "      c = make_uint4(code4(lut, x.x), code4(lut, x.y), code4(lut, x.z), code4(lut, x.w));",
                   "      c = x;")],
    "rb_ntload": [("kernels_http_raw.hip", "      if (!pad && sub <= units) x = rec16[(size_t)rs + sub];",
                   "      if (!pad && sub <= units) x = ld_nt16(rec16 + (size_t)rs + sub);")],
    "rb_ntstore": [("kernels_http_raw.hip", "        reinterpret_cast<uint4*>(tb + 512)[(size_t)u * 64 + s] = c;",
                    "        st_nt16(reinterpret_cast<uint4*>(tb + 512) + (size_t)u * 64 + s, c);")],
    # the tile walkers' lane offset as the kernel's (spilled) copy instead of recomputed
    "h_nolanenow": [('  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\\n\\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));',
                     "  l = threadIdx.x & 63;")],
    # measuring device (verdicts land in order[] in slot order, out[] is not
    # written): raw-mode http_kernel without the verdict scatter
    "h_noscatter": [("      const uint32_t r = order[slot];\n      if (r < nout) {\n        out[r] = (uint8_t)v;",
                     "      const uint32_t r = order[slot];\n      if (r < nout) {\n        const_cast<uint32_t*>(order)[slot] = v;")],
    # 5 KiB stages with the scan capped at 128 VGPRs (4 waves per SIMD when
    # LDS allows: 40.9 KB per block at config 5)
    "raw_s5k_w4": _rs(5120) + [("kernels_http_raw.hip",
                                "__global__ __launch_bounds__(kRawThreads) void raw_scan_kernel(",
                                "__global__ __launch_bounds__(kRawThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void raw_scan_kernel(")],
    "rank_u4": [("kernels_http_raw.hip", "constexpr uint32_t kRankU = 8;", "constexpr uint32_t kRankU = 4;")],
    "raw_ldscodes": [("kernels_http_raw.hip", "return (size_t)R.nprogs * 256 <= 4 * 1024; }",
                      "return (size_t)R.nprogs * 256 <= 32 * 1024; }")],
    # ipcache: addresses per lane (v4, v6)
    "ipc_v6u4": [("kernels_ipcache.hip", "constexpr uint32_t kIpcV4 = 4, kIpcV6 = 2;",
                  "constexpr uint32_t kIpcV4 = 4, kIpcV6 = 4;")],
    "ipc_v4u8": [("kernels_ipcache.hip", "constexpr uint32_t kIpcV4 = 4, kIpcV6 = 2;",
                  "constexpr uint32_t kIpcV4 = 8, kIpcV6 = 2;")],
    # round 5 measuring devices on the class-mode walker (verdicts meaningless;
    # every LDS address stays inside the block or reads LDS out of range as 0):
    # the DFA step without its LDS read (same VALU count), and no walk at all
    # (the unit loads stay: the step's asm still consumes every unit word)
    "h_nolds": [('"\\n\\tds_read_b32 %0, %0\\n\\t"', '"\\n\\tv_mov_b32 %0, %3\\n\\t"')],
    "h_nowalk": [('  if (B == 0) CG_CLS_STEP("BYTE_0");',
                  '  if (true) {\n    asm volatile("v_mov_b32 %0, %1" : "=v"(nx) : "v"(st), "v"(w));\n    return nx;\n  }\n'
                  '  if (B == 0) CG_CLS_STEP("BYTE_0");')],
    # two tiles per wave, one request of each per lane, two LDS chains
    # (lds_cls_step2); h_pair_w1: a one-unit rolling window per chain
    "h_pair": [("constexpr bool kPairTiles = false;", "constexpr bool kPairTiles = true;")],
    "h_pair_w1": [("constexpr bool kPairTiles = false;", "constexpr bool kPairTiles = true;"),
                  ("  constexpr int kW = N < 2 ? (N > 0 ? N : 1) : 2;", "  constexpr int kW = 1;")],
    # measuring device: the device-layout scan's string units written
    # uncoded (no per-byte code-map loads; verdicts meaningless)
    "rawdl_nocode": [("raw_emit.h", "CG_HD inline uint32_t code4(const uint8_t* lut, uint32_t q) {\n  return",
                      "CG_HD inline uint32_t code4(const uint8_t* lut, uint32_t q) {\n  return q; return"),
                     ("kernels_http_raw.hip", "#include <hip/hip_runtime.h>", "#include <hip/hip_runtime.h>")],
    # measuring devices: the device-layout scan without its string units
    # (no code-map loads, no unit stores), and without the slot protocol (a
    # slot computed from the request index: no atomics, no directory polls)
    "rawdl_noemit": [("kernels_http_raw.hip", "        emit_stage(R, stage, hs, sp, kRawThreads, P, last, o);",
                      "        (void)o;")],
    "rawdl_noslot": [("kernels_http_raw.hip",
                      "    const RawSlot sl = raw_slot(L, want, raw_vkey(L, group_of(R, prog) * kRawUnits + units, blockIdx.x), prog);",
                      "    const uint32_t tfake = (uint32_t)((i >> 6) % L.maxchunks);\n"
                      "    const RawSlot sl{L.tiles + (size_t)tfake * (kRawTileGran * 512), tfake, (uint32_t)(i & 63), want};")],
    # the device-layout scan's string units stored nontemporal (verdicts
    # valid), and as a measuring device without the unit stores (the units'
    # bytes still gathered; verdicts meaningless, memory-safe)
    "rawdl_ntunits": [("raw_emit.h", "    *dst = kCode ? make_uint4(code4(lut, w0), code4(lut, w1), code4(lut, w2), code4(lut, w3)) : make_uint4(w0, w1, w2, w3);",
                       "    { typedef unsigned int v4u __attribute__((ext_vector_type(4))); __builtin_nontemporal_store(v4u{w0, w1, w2, w3}, reinterpret_cast<v4u*>(dst)); }"),
                      ("raw_emit.h", "    *dst = make_uint4(keep(c(w0), 0), keep(c(w1), 4), keep(c(w2), 8), keep(c(w3), 12));",
                       "    { typedef unsigned int v4u __attribute__((ext_vector_type(4))); __builtin_nontemporal_store(v4u{keep(c(w0), 0), keep(c(w1), 4), keep(c(w2), 8), keep(c(w3), 12)}, reinterpret_cast<v4u*>(dst)); }"),
                      ("kernels_http_raw.hip", "#include <hip/hip_runtime.h>", "#include <hip/hip_runtime.h>")],
    "rawdl_nounitst": [("raw_emit.h", "    *dst = kCode ? make_uint4(code4(lut, w0), code4(lut, w1), code4(lut, w2), code4(lut, w3)) : make_uint4(w0, w1, w2, w3);",
                        "    asm volatile(\"\" ::\"v\"(w0), \"v\"(w1), \"v\"(w2), \"v\"(w3));"),
                       ("raw_emit.h", "    *dst = make_uint4(keep(c(w0), 0), keep(c(w1), 4), keep(c(w2), 8), keep(c(w3), 12));",
                        "    asm volatile(\"\" ::\"v\"(keep(c(w0), 0)), \"v\"(keep(c(w1), 4)), \"v\"(keep(c(w2), 8)), \"v\"(keep(c(w3), 12)));"),
                       ("kernels_http_raw.hip", "#include <hip/hip_runtime.h>", "#include <hip/hip_runtime.h>")],
    # a wave issuing its tile's loads (window + next tile's head) at raised
    # priority, so the loads leave before other waves' walk steps
    "h_prio": [("  const uint2 meta = cur.meta;\n", "  __builtin_amdgcn_s_setprio(3);\n  const uint2 meta = cur.meta;\n"),
               ("  if (has_next) tile_prefetch(trn, nunits, lane, nxt);\n  __builtin_amdgcn_sched_barrier(0);",
                "  if (has_next) tile_prefetch(trn, nunits, lane, nxt);\n  __builtin_amdgcn_s_setprio(0);\n  __builtin_amdgcn_sched_barrier(0);")],
    # 4 waves per SIMD (128 VGPRs, one 1024-thread workgroup per CU): the
    # registers spent on a second chain (pairs) and / or deeper prefetch
    "h_pair_w4": [("constexpr bool kPairTiles = false;", "constexpr bool kPairTiles = true;"),
                  ("constexpr int kHttpWaves = 8;", "constexpr int kHttpWaves = 4;")],
    "h_pair_w4_pre2": [("constexpr bool kPairTiles = false;", "constexpr bool kPairTiles = true;"),
                       ("constexpr int kHttpWaves = 8;", "constexpr int kHttpWaves = 4;"),
                       ("constexpr int kPre = 1;", "constexpr int kPre = 2;")],
    "h_w4_pre4": [("constexpr int kHttpWaves = 8;", "constexpr int kHttpWaves = 4;"),
                  ("constexpr int kPre = 1;", "constexpr int kPre = 4;")],
    # the scans at 512 threads per workgroup (spans / tables amortized over 8
    # waves) with 5 KiB stages: 2 workgroups = 4 waves per SIMD at config 5;
    # and 5 KiB stages alone (256 threads)
    "rawdl_t512_s5k": [("dev_types.h", "constexpr uint32_t kRawScanThreads = 256;",
                        "constexpr uint32_t kRawScanThreads = 512;"),
                       ("kernels_http_raw.hip", "constexpr uint32_t kStage = 6144;", "constexpr uint32_t kStage = 5120;"),
                       ("http_raw.cc", "#include", "#include")],
    "rawdl_s5k": _rs(5120),
    # measuring devices (verdict counters / rows wrong, verdicts still
    # written): no per-rule hit counting, no remote-identity row lookup
    "h_nohits": [("  count_hits(T, pg, hit, s_hits, lane);\n", "")],
    "h_norow": [("const uint32_t row = remote_row(blk, pg, meta.x);", "const uint32_t row = pg.default_remote;")],
    # verdict bytes stored nontemporal (slot-order batches)
    "h_ntout": [("      out[slot] = (uint8_t)v;\n", "      __builtin_nontemporal_store((uint8_t)v, out + slot);\n")],
    # Kafka verdict kernel: requests per lane per iteration (queue sized with it)
    "kv_r2": [("kernels.hip", "constexpr uint32_t kKafkaReqs = 4;", "constexpr uint32_t kKafkaReqs = 2;")],
    "kv_r8": [("kernels.hip", "constexpr uint32_t kKafkaReqs = 4;", "constexpr uint32_t kKafkaReqs = 8;")],
    # chunks per dealt run (program block restaged once per run)
    "h_deal8": [("constexpr uint32_t kDealRun = 4;", "constexpr uint32_t kDealRun = 8;")],
    "h_deal2": [("constexpr uint32_t kDealRun = 4;", "constexpr uint32_t kDealRun = 2;")],
})


def build_variant(name, subs):
    """subs: (old, new) pairs on kernels_http.hip, or (file, old, new) on any
    csrc/ source; the changed sources are compiled into a private library."""
    OUT.mkdir(exist_ok=True)
    files = {}
    for sub in subs:
        fn, a, b = sub if len(sub) == 3 else ("kernels_http.hip", *sub)
        src = files.get(fn) or (B.CSRC / fn).read_text()
        assert a in src, (name, fn, a)
        files[fn] = src.replace(a, b)
    if not any(fn.endswith(".hip") for fn in files) and not name.startswith(("l4_", "lpm_")):
        files["kernels_kafka.hip" if name.startswith("kw_") else "kernels_http.hip"] = \
            (B.CSRC / ("kernels_kafka.hip" if name.startswith("kw_") else "kernels_http.hip")).read_text()
    objs = []
    # a variant's sources go to their own directory: a changed header there
    # is found first by the changed sources' quote includes
    vdir = OUT / name
    vdir.mkdir(exist_ok=True)
    # every header goes there too (a changed one included from an unchanged
    # header would otherwise be found twice under #pragma once)
    for h in B.CSRC.glob("*.h"):
        if h.name not in files:
            (vdir / h.name).write_text(h.read_text().replace('"../../include/', f'"{ROOT}/include/'))
    for fn, src in files.items():
        (vdir / fn).write_text(src.replace('"../../include/', f'"{ROOT}/include/'))
    for fn in files:
        if fn.endswith(".h"):
            continue
        obj = vdir / f"{fn}.o"
        cmd = [B.HIPCC, *B._flags(fn), "-I", str(B.CSRC), "-I", str(ROOT / "include"), "-c", str(vdir / fn), "-o",
               str(obj)]
        subprocess.run(cmd, check=True)
        objs.append(obj)
    others = [B.BUILD / (s + ".o") for s in B.SOURCES if s not in files]
    lib = OUT / f"lib_{name}.so"
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *map(str, others), *map(str, objs),
                    "-o", str(lib), "-lpthread", "-lz", "-lhsa-runtime64"], check=True)
    print("built", lib)


if __name__ == "__main__":
    B.build(verbose=False)
    names = sys.argv[2:] or list(VARIANTS)
    for n in names:
        build_variant(n, VARIANTS[n])
