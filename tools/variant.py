#!/usr/bin/env python3
"""Experiment builds from a patched COPY of the kernel source (round 4: the product source carries no experiment
macros).  A patch is a list of (old, new) string replacements applied to csrc/h12env.hip in a scratch tree under
tools/_variants/<tag>/ (with include/ beside it, so the relative includes resolve); the library is
tools/_variants/lib_<tag>.so, loaded with H12ENV_LIB=... by bench.py / tools/phase_profile.py.

    python tools/variant.py <tag> [--profile]      # builds the variant named <tag> from PATCHES below
    python tools/variant.py r5prev@HEAD            # the committed kernel, unpatched (A/B baseline)
"""
from __future__ import annotations

import argparse
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "h1v2-isaac_amd"))

# The recorded round-4 experiments were written against the round-4 kernel (commit R4_BASE): they are applied to that
# commit's sources (git show), so they stay reproducible while the product kernel moves on.  Experiments against the
# current sources go into PATCHES_HEAD.
R4_BASE = "787ede1"

PATCHES = {
    # the helper waves' shifted-row stores during the physics loop dropped (timing only: the rows are wrong)
    "no_early": [("  for (int k = k0; k < k1; ++k) {\n    const int j = t + k * nt;",
                  "  for (int k = k0; k < k0; ++k) {\n    const int j = t + k * nt;")],
    # the Rough observation's height scan without its heightfield gathers (timing only: the scan reads 0)
    "scan_nogather": [("      hz = ground(P, px + cy * xl - sy * yl, py + sy * xl + cy * yl, gx, gy);",
                       "      hz = 0.f * (px + cy * xl - sy * yl) * (py + sy * xl + cy * yl); gx = gy = 0.f;")],
    # probe: 300 VALU of dependent dummy work in the self-contact wave before R1 (its slack there)
    "self_slack150": [("      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];",
                        "      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n" + '      {  // probe: N dependent FMAs of dummy work in the self-contact wave before R1 (its slack there)\n        float d0 = p[0], d1 = p[1];\n        for (int i = 0; i < NDUMMY; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile("" :: "v"(d0), "v"(d1));\n      }\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];'.replace("NDUMMY", "150"))],
    # probe: 600 VALU of dependent dummy work in the self-contact wave before R1 (its slack there)
    "self_slack300": [("      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];",
                        "      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n" + '      {  // probe: N dependent FMAs of dummy work in the self-contact wave before R1 (its slack there)\n        float d0 = p[0], d1 = p[1];\n        for (int i = 0; i < NDUMMY; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile("" :: "v"(d0), "v"(d1));\n      }\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];'.replace("NDUMMY", "300"))],
    # probe: 1200 VALU of dependent dummy work in the self-contact wave before R1 (its slack there)
    "self_slack600": [("      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];",
                        "      act = self_stage(P, leg, lg.mud, Rk, pk, v[3], R, p, v[5]);\n" + '      {  // probe: N dependent FMAs of dummy work in the self-contact wave before R1 (its slack there)\n        float d0 = p[0], d1 = p[1];\n        for (int i = 0; i < NDUMMY; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile("" :: "v"(d0), "v"(d1));\n      }\n    }\n    __syncthreads();  // R1\n    if (active) {\n      float w[12];'.replace("NDUMMY", "600"))],
    # probe: 600 VALU of dependent dummy work in the helper wave before R1 (its slack there)
    "helper_slack300": [("      if constexpr (Feat<K>::terrain) helper_torso<K>(P, l, leg, b, vb, R0, pb0, org);\n    }\n    __syncthreads();  // R1",
                         "      if constexpr (Feat<K>::terrain) helper_torso<K>(P, l, leg, b, vb, R0, pb0, org);\n      {\n        float d0 = p[0], d1 = p[1];\n        for (int i = 0; i < 300; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile(\"\" :: \"v\"(d0), \"v\"(d1));\n      }\n    }\n    __syncthreads();  // R1")],
    # the state write-back dropped (timing only: the state never advances)
    "no_store": [("    store_env<K>(P, W, e, leg, s);\n    PH(7);", "    PH(7);")],
    # static probe: the MDP state loaded after the physics loop (register pressure in the loop; Flat only -- the
    # terrain origin is loaded before the loop as well)
    "mdp_late": [("    load_mdp<K>(P, W, e, leg, s);\n    PH(0);",
                  "    for (int i = 0; i < 3; ++i) s.origin[i] = Feat<K>::terrain ? ldf(W, H12_F_ORIGIN + i, e) : 0.f;\n    PH(0);"),
                 ("    PH(1);\n    // ContactSensor._update_buffers_impl", "    PH(1);\n    load_mdp<K>(P, W, e, leg, s);\n    // ContactSensor._update_buffers_impl")],
    # the link velocities parked in the joint-terms LDS slot (free after the physics wave has read it at R1) and read
    # back before the base pair sum for pass 3
    "v_lds": [("    knee_pz = jt[26];\n  } else {",
               "    knee_pz = jt[26];\n    put4(help_lds().jt, threadIdx.x, &v[0][0], 9);\n  } else {"),
              ("  // ---- pair sum in fixed (left + right) order: both lanes hold bit-identical base quantities\n",
               "  // ---- pair sum in fixed (left + right) order: both lanes hold bit-identical base quantities\n"
               "  if constexpr (HW) get4(help_lds().jt, threadIdx.x, &v[0][0], 9);\n")],
    # probes: 300 VALU of dependent dummy work in the R1 -> R2 window of the self-contact / helper wave
    "self_r2slack300": [("      put4(H.selfw, l, w, 3);\n    }",
                         "      put4(H.selfw, l, w, 3);\n      {\n        float d0 = w[0], d1 = w[1];\n        for (int i = 0; i < 150; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile(\"\" :: \"v\"(d0), \"v\"(d1));\n      }\n    }")],
    "helper_r2slack300": [("      put4(H.bias, l, o, 11);\n",
                           "      put4(H.bias, l, o, 11);\n" + "      {\n        float d0 = w[0], d1 = w[1];\n        for (int i = 0; i < 150; ++i) { d0 = __builtin_fmaf(d0, 0.999f, d1); d1 = __builtin_fmaf(d1, 1.001f, d0); }\n        asm volatile(\"\" :: \"v\"(d0), \"v\"(d1));\n      }\n".replace("w[0]", "o[0]").replace("w[1]", "o[1]"))],
    # 16 envs per block (256 blocks at 4096 envs: one per CU), the upper half of every 64-lane wave idle; a correct
    # build (the parity tests run on it with H12ENV_LIB)
    "epb16": [("constexpr int ENVS_PER_BLOCK = 32;", "constexpr int ENVS_PER_BLOCK = 16;"),
              ("  const bool active = step_block() * ENVS_PER_BLOCK + (l >> 1) < n;",
               "  const bool active = (l >> 1) < ENVS_PER_BLOCK && step_block() * ENVS_PER_BLOCK + (l >> 1) < n;", 2),
              ("  const int e = e0 + lane_pair;",
               "  const int e = lane_pair < ENVS_PER_BLOCK ? e0 + lane_pair : 0x3fffffff;", 3),
              ("  const int e = blockIdx.x * ENVS_PER_BLOCK + lane_pair;",
               "  const int e = lane_pair < ENVS_PER_BLOCK ? blockIdx.x * ENVS_PER_BLOCK + lane_pair : 0x3fffffff;"),
              ("  const int e = blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1);",
               "  const int e = (threadIdx.x >> 1) < ENVS_PER_BLOCK ? blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1) "
               ": 0x3fffffff;", 2)],
}
PATCHES_HEAD: dict = {
    # round 6: 16 envs per block on the current kernel (256 blocks at 4096 envs, one per CU, the upper half of every wave
    # idle): round 4's epb16 re-expressed for the round-5 kernel (four waves, shared self-contact jobs, fused rows)
    "epb16h": [("constexpr int ENVS_PER_BLOCK = 32;", "constexpr int ENVS_PER_BLOCK = 16;"),
               ("  const bool active = step_block() * ENVS_PER_BLOCK + (l >> 1) < n;",
                "  const bool active = (l >> 1) < ENVS_PER_BLOCK && step_block() * ENVS_PER_BLOCK + (l >> 1) < n;", 3),
               ("      const int he = step_block() * ENVS_PER_BLOCK + (hl >> 1);",
                "      const int he = (hl >> 1) < ENVS_PER_BLOCK ? step_block() * ENVS_PER_BLOCK + (hl >> 1) : 0x3fffffff;"),
               ("  const int e = e0 + lane_pair;",
                "  const int e = lane_pair < ENVS_PER_BLOCK ? e0 + lane_pair : 0x3fffffff;", 3),
               ("  const int e = blockIdx.x * ENVS_PER_BLOCK + lane_pair;",
                "  const int e = lane_pair < ENVS_PER_BLOCK ? blockIdx.x * ENVS_PER_BLOCK + lane_pair : 0x3fffffff;"),
               ("  const int e = blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1);",
                "  const int e = (threadIdx.x >> 1) < ENVS_PER_BLOCK ? blockIdx.x * ENVS_PER_BLOCK + (threadIdx.x >> 1) "
                ": 0x3fffffff;", 2)],
    # round 6 timing probe (results wrong): the physics wave's three link chains (inertia chain before R2, bias-force
    # chain and pass 3 after it) over links 3-5 only -- half of the chains' work removed, the best case of splitting
    # them over two lanes per leg with free exchanges.  "_h" = on the 32-env kernel, "epb16h_half" = on epb16h
    "chain_half": [("  link_ia<2, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);\n"
                    "  link_ia<1, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);\n"
                    "  link_ia<0, true>(P, lg, cs, v, ick, knee_pz, dl, IA, U, Dinv, Ic, h);\n", ""),
                   ("    link_p_pk<2>(cs, U, Dinv, tau, pb, p, u);\n    link_p_pk<1>(cs, U, Dinv, tau, pb, p, u);\n"
                    "    link_p_pk<0>(cs, U, Dinv, tau, pb, p, u);\n", ""),
                   ("  link_pass3_pk<0>(cs, U, Dinv, u, ap, qdd);\n  link_pass3_pk<1>(cs, U, Dinv, u, ap, qdd);\n"
                    "  link_pass3_pk<2>(cs, U, Dinv, u, ap, qdd);\n", "  qdd[0] = qdd[1] = qdd[2] = 0.f;\n")],
    # probe: the episode sums loaded after the helper wave's loop (is their load the helper's delay at the first S?)
    "epsum_late": [("      if (he < W.n) load_epsum<K>(P, W, he, ep);\n      helper_wave<K>(P, W.n, nsteps, (uint32_t)(A.env_offset + he), A.lo, A.hi, fc);",
                    "      helper_wave<K>(P, W.n, nsteps, (uint32_t)(A.env_offset + he), A.lo, A.hi, fc);\n      if (he < W.n) load_epsum<K>(P, W, he, ep);")],
    # the knee capsule's ground contact on the self-contact wave (round 5 experiment: that wave became the last at R1,
    # -1.5 %, profiles/r5/r5q_*)
    "knee_self": [("constexpr bool KNEE_ON_SELF = false;", "constexpr bool KNEE_ON_SELF = true;")],
    # the helper waves' shifted-row stores with the default (write-back) policy instead of nt: the newest-slot floats
    # written after barrier F then merge into the L2 lines of their rows (round 4's +1.29 MB of partial-line writes)
    "rows_wb": [("""                                         __builtin_amdgcn_make_buffer_rsrc(dst, 0, -1, 0x00020000), j * 16, 0,
                                         ST_POL);""", """                                         __builtin_amdgcn_make_buffer_rsrc(dst, 0, -1, 0x00020000), j * 16, 0,
                                         0);""")],
}
PATCHES_HEAD["epb16h_half"] = PATCHES_HEAD["epb16h"] + PATCHES_HEAD["chain_half"]
# round 6 timing probe: epb16h_half plus the lane exchanges a two-lanes-per-leg split puts on the chains, as identity
# double swaps (two dependent DPP lane swaps) of the chains' own values -- per link 16 swaps in the inertia chain (U, C,
# the shift correction: ~15 values a split hands over once each), 4 in the bias chain, 6 in pass 3
_XS = ("H12_DEV float xs2(float x) { return pair_swap(pair_swap(x)); }\n"
       "template <int LINK, bool AV = false, typename UT>\nH12_DEV void link_ia(")
PATCHES_HEAD["epb16h_halfx"] = PATCHES_HEAD["epb16h_half"] + [
    ("template <int LINK, bool AV = false, typename UT>\nH12_DEV void link_ia(", _XS),
    ("  ai_rotate<A>(IA, cs[LINK][0], cs[LINK][1]);\n  ai_shift(IA, h12m::R[LINK]);\n",
     "  ai_rotate<A>(IA, cs[LINK][0], cs[LINK][1]);\n"
     "  for (int k = 0; k < 3; ++k) IA.C[k] = xs2(IA.C[k]);\n"
     "  ai_shift(IA, h12m::R[LINK]);\n"
     "  for (int k = 0; k < 2; ++k) IA.A[k] = xs2(IA.A[k]);\n"),
    ("  float D = IA.A[A] + h12m::ARM[LINK]",
     "  for (int k = 0; k < 3; ++k) Ua[k] = xs2(Ua[k]);\n  float D = IA.A[A] + h12m::ARM[LINK]"),
    ("  const float ud = uu * Dinv[LINK];\n  f32x2 pa[3], q[3];\n",
     "  const float ud = xs2(xs2(uu) * Dinv[LINK]);\n  f32x2 pa[3], q[3];\n"),
    ("  const float x = (u[LINK] - (ua.x + ua.y)) * Dinv[LINK];\n",
     "  const float x = xs2(xs2(u[LINK] - (xs2(ua.x) + ua.y)) * Dinv[LINK]);\n"),
]
# round 6 timing probe (results wrong): the self-contact pair jobs' LDS float atomics (12 per contact point, up to 16 lanes
# of one env on the same address in the foot-foot passes) replaced by consuming the values -- what the atomics' address
# conflicts cost the candidate blocks
PATCHES_HEAD["self_noatomic"] = [
    ("        lds_add(al(a), F[a]); lds_add(al(3 + a), m[a]);\n        lds_add(ar(a), -F[a]); lds_add(ar(3 + a), -m[a]);\n",
     "        asm volatile(\"\" :: \"v\"(F[a]), \"v\"(m[a]));\n")]
# round 6 bias elimination (correct results, slower math): one single-instruction operation of the kernel replaced by its
# correctly rounded form, to see which one carries the signed bias left after the fsincos fix (tools/bias_probe.py)
_ACC = {"acc_rsq": "#define __builtin_amdgcn_rsqf(x) (1.0f / __builtin_sqrtf(x))\n",
        "acc_rcp": "#define frcp(x) (1.0f / (x))\n",
        "acc_sqrt": "#define fsqrt(x) __builtin_sqrtf(x)\n",
        "acc_pre": ("H12_DEV void fsincos_acc(float x, float* s, float* c) {\n"
                    "  const float y = __builtin_fmaf(x, 0.15915493667125702f, x * 6.4206382e-09f);\n"
                    "  const float sv = __builtin_amdgcn_sinf(y), cv = __builtin_amdgcn_cosf(y);\n"
                    "  const float d = __builtin_fmaf(cv, cv, __builtin_fmaf(sv, sv, -1.f));\n"
                    "  *s = __builtin_fmaf(sv, -0.5f * d, sv);\n  *c = __builtin_fmaf(cv, -0.5f * d, cv);\n}\n"
                    "#define fsincos(x, s, c) fsincos_acc(x, s, c)\n")}
for _k, _v in _ACC.items():
    PATCHES_HEAD[_k] = [("using namespace h12;\n", "using namespace h12;\n" + _v)]
PATCHES_HEAD["acc_all"] = [("using namespace h12;\n", "using namespace h12;\n" + "".join(_ACC.values()))]
# round 6 block-tail probes (timing only, results wrong): the flat torso contact off the helper wave; the helper waves'
# drain of the row LDS-DMA before barrier R2 of inner step 1 skipped
PATCHES_HEAD["no_torso"] = [("      if constexpr (!Feat<K>::terrain) helper_torso<K>(P, l, leg, b, vb, R0, pb0, org);\n", "")]
PATCHES_HEAD["no_drain"] = [("  if (f.on && it == 1) __builtin_amdgcn_s_waitcnt(0);", "  (void)f; (void)it;")]
# round 6 private-segment fix B (measured, not kept: profiles/r6/not_kept/private_segment_ab.txt): the StepArgs output
# pointers re-read after the physics loop through an opaque kernarg-segment pointer, so the entry's 16-dword StepArgs
# s_load is not live across the loop; and the probe on top of it (timing only): a never-taken dynamically indexed
# private array that gives the step kernel a private segment again, with real scratch instructions
_LATE = """constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
constexpr size_t STEP_ARGS_KOFF = align_up(align_up(sizeof(KParams), alignof(Workspace)) + sizeof(Workspace), alignof(StepArgs));
H12_DEV const __attribute__((address_space(4))) StepArgs& late_step_args() {
  auto p = (const __attribute__((address_space(4))) StepArgs*)(
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() + STEP_ARGS_KOFF);
  asm volatile("" : "+s"(p));
  return *p;
}
"""
PATCHES_HEAD["late_step_args"] = [
    ("H12_DEV void kernarg_warm() {", _LATE + "H12_DEV void kernarg_warm() {"),
    ("      if (he < W.n) {\n        if (hleg == 0) A.rew[he] = r;", "      const auto& AL = late_step_args();\n"
     "      if (he < W.n) {\n        if (hleg == 0) AL.rew[he] = r;"),
    ("      if (lv) A.log_part[(size_t)v * gridDim.x + blockIdx.x] = lacc;",
     "      if (lv) AL.log_part[(size_t)v * gridDim.x + blockIdx.x] = lacc;"),
    ("    if (leg == 0) {\n      A.term[e] = (uint8_t)term;\n      A.trunc[e] = (uint8_t)tout;\n    }\n"
     "    if (A.applied_torque)\n      for (int k = 0; k < NL; ++k) A.applied_torque[",
     "    const auto& AL = late_step_args();\n    if (leg == 0) {\n      AL.term[e] = (uint8_t)term;\n"
     "      AL.trunc[e] = (uint8_t)tout;\n    }\n    if (AL.applied_torque)\n"
     "      for (int k = 0; k < NL; ++k) AL.applied_torque["),
    ("    if (A.foot_force) A.foot_force[2 * e + leg] = flast_foot;",
     "    if (AL.foot_force) AL.foot_force[2 * e + leg] = flast_foot;")]
PATCHES_HEAD["scratch_pad"] = PATCHES_HEAD["late_step_args"] + [
    ("  H12_BW_KSTART();\n  kernarg_warm();\n",
     "  H12_BW_KSTART();\n  kernarg_warm();\n  if (P.dbg_norel == 0x5eed) {\n    volatile int pad[17];\n"
     "    pad[threadIdx.x % 17] = (int)threadIdx.x;\n    P.diag[0] = pad[(threadIdx.x + 1) % 17];\n  }\n")]
# round 6 CaT in-kernel probabilities, timing probes (results wrong): the helper waves skip the wait for the fold's
# epoch; or they wait but skip the per-env probability chain after it
PATCHES_HEAD["cat_nowait"] = [("    while (((w = ld_sc1(pub)) >> 32) == e0 && ++k < CAT_WAIT_POLLS) __builtin_amdgcn_s_sleep(2);\n",
                               "    w = ld_sc1(pub); (void)e0;\n")]
PATCHES_HEAD["cat_nochain"] = [("  if (on) keep = cat_prob_env(W, A, he, j, reset, vs, vp, src, rinv, lg);\n",
                                "  (void)vs; (void)vp; (void)src; (void)reset;\n")]
# ... and the floor: no hand-off, fold, wait or probabilities at all (the constraint values are still computed)
PATCHES_HEAD["cat_floor"] = [
    ("      const bool cat_w = Feat<K>::ext && P.cat && threadIdx.x < 3 * BLOCK;", "      const bool cat_w = false;"),
    ("      if (Feat<K>::ext && A.cat_inline) r *= cat_prob_inline(W, A, he, hl >> 1, cat_on, hreset, cvs, cvp);\n", "")]
# ... the fold after barrier F (the non-last blocks do not wait for their add's return before F), before the rows;
# and the hand-off without the still envs' no_move row stores (results wrong: timing of that part)
PATCHES_HEAD["cat_fold_after_f"] = [
    ("            if (cat_is_last(cat_old)) cat_fold(P, W.n, true);\n", ""),
    ("        __syncthreads();  // F\n        fuse_late(P, A, fc, W.n, ft, fnt);\n      } else if (cat_w) {",
     "        __syncthreads();  // F\n        if (cat_w && cat_inl && cat_is_last(cat_old)) cat_fold(P, W.n, true);\n"
     "        fuse_late(P, A, fc, W.n, ft, fnt);\n      } else if (cat_w) {")]
PATCHES_HEAD["cat_no_nmrows"] = [("        st_sc1(&P.cscr[(size_t)(NM0 + k) * n + e], cv[NM0 + k][j]);\n", "        (void)e;\n")]
# round 6 side-rod cost probe (timing only, results wrong): every sole_contacts_flat call evaluates one more sphere (its
# last one again) -- the work the side rods' front ends would add to each of the two sole waves
PATCHES_HEAD["siderod_probe"] = [("#pragma unroll\n  for (int q = Q0; q < Q1; ++q) {\n    float r[3];\n",
                                  "#pragma unroll\n  for (int qq = Q0; qq <= Q1; ++qq) {\n    const int q = qq < Q1 ? qq : Q1 - 1;\n"
                                  "    float r[3];\n")]
# round 6 NaN hunt (rsl / cat at 8192 envs, tools/probe/determinism.py): the self-contact wave's pass 1 with the corrected
# joint sin / cos; the radial correction off everywhere
PATCHES_HEAD["nan_selfcorr"] = [("leg_pass1<K, true>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p, true);",
                                 "leg_pass1<K, false>(leg, b, lg, org, R0, vb, pb0, cs, v, Rk, pk, R, p, true);")]
PATCHES_HEAD["nan_nocorr"] = [("using namespace h12;\n", "using namespace h12;\n#define fsincos(x, s, c) fsincos_hw(x, s, c)\n")]
ALL = {**{k: (R4_BASE, v) for k, v in PATCHES.items()}, **{k: (None, v) for k, v in PATCHES_HEAD.items()}}
# the CaT probes were measured on commit 306df83's kernel (profiles/r6/cat_inline_ab.txt)
for _k in ("cat_nowait", "cat_nochain", "cat_floor", "cat_fold_after_f", "cat_no_nmrows"):
    ALL[_k] = ("306df83", ALL[_k][1])
SOURCES = ("h1v2-isaac_amd/csrc/h12env.hip", "h1v2-isaac_amd/csrc/h12_math.h", "h1v2-isaac_amd/csrc/h12_model_gen.h",
           "include/h12env.h")


def source_at(rev: str | None, rel: str) -> str:
    """A kernel source file of the working tree (rev None) or of git revision rev."""
    if rev is None:
        return (ROOT / rel).read_text()
    return subprocess.run(["git", "show", f"{rev}:{rel}"], cwd=ROOT, check=True, capture_output=True, text=True).stdout


def patched(tag: str) -> tuple[str, str]:
    """(original, patched) h12env.hip of variant tag"""
    rev, patches = ALL[tag] if tag in ALL else (tag.split("@", 1)[1] or None, [])
    src = orig = source_at(rev, SOURCES[0])
    for old, new, *cnt in patches:  # (old, new[, expected number of matches, default 1])
        want = cnt[0] if cnt else 1
        if src.count(old) != want:
            raise SystemExit(f"patch {tag!r}: {old[:60]!r} matches {src.count(old)} times, not {want}")
        src = src.replace(old, new)
    return orig, src


def build(tag: str, profile: bool, isa: bool = False, light: bool = False) -> Path:
    from h12env.build import ARCH, hipcc

    rev = ALL[tag][0] if tag in ALL else (tag.split("@", 1)[1] or None)
    _, src = patched(tag)
    tag = tag.split("@", 1)[0]
    top = ROOT / "tools" / "_variants" / tag
    if top.exists():
        shutil.rmtree(top)
    csrc = top / "a" / "csrc"
    csrc.mkdir(parents=True)
    (top / "include").mkdir()
    for rel in SOURCES[1:]:
        dst = top / "include" / Path(rel).name if rel.startswith("include/") else csrc / Path(rel).name
        dst.write_text(source_at(rev, rel))
    (csrc / "h12env.hip").write_text(src)
    out = ROOT / "tools" / "_variants" / f"lib_{tag}.so"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fno-slp-vectorize", "-Xarch_device",
           "-ffinite-math-only", "-Xarch_device", "-fno-signed-zeros", "-fPIC", "-shared", "-Wno-unused-function",
           *(["-DH12_PHASE_PROFILE"] if profile or light else []), *(["-DH12_PHASE_LIGHT"] if light else []),
           *(["-save-temps"] if isa else []), "-o", str(out),
           str(csrc / "h12env.hip")]
    subprocess.run(cmd, check=True, cwd=top)
    if isa:  # the Flat step kernel's static report (tools/kernel_isa.py), as for the product
        sys.path.insert(0, str(ROOT / "tools"))
        import kernel_isa

        text = sorted(top.glob(f"*{ARCH}*.s"))[0].read_text()
        name = "_ZN12_GLOBAL__N_111step_kernelILi0EEEvNS_7KParamsENS_9WorkspaceENS_8StepArgsE"
        md = kernel_isa.metadata(text)[name]
        r = kernel_isa.report(text, name)
        print("vgpr", md.get("vgpr_count"), "agpr", md.get("agpr_count"), "valu", r["valu"], "accvgpr", r["accvgpr"])
        for lp in r["loops"]:
            if lp[1] > 2000:
                print("  loop", lp)
    shutil.rmtree(top)
    print("built", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", help=f"one of {sorted(ALL)}, or <name>@<git revision>: that revision's unpatched "
                    "sources as tools/_variants/lib_<name>.so (the A/B baseline; <name>@ alone: the working tree's)")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--light", action="store_true", help="the light-stamp profile build (tools/phase_profile.py --tag <tag>)")
    ap.add_argument("--isa", action="store_true", help="print the Flat step kernel's static ISA report")
    a = ap.parse_args()
    build(a.tag, a.profile, a.isa, a.light)
