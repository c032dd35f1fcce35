// pt_tool_hooks.h — measurement scaffolding for tool builds of libptamd.so (never the product).
//
// The product kernels carry PT_HOOK(NAME, ...) call sites that expand to nothing.  A tool build
// (tools/mkvar.sh "-DPT_TOOLS -DPT_DUP=N" or "-DPT_TOOLS -DPT_PROBE_EXTRA_LOAD") includes this
// header instead (pt_device.h), and the hooks below do extra work whose cost a PMC / timing A/B
// then measures:
//
//   PT_DUP=1..5  one section executed twice, the duplicate's result discarded (its inputs are
//                perturbed by +0 so it is not folded into the first): the difference in
//                SQ_INSTS_VALU is the section's count (tools/valu_attrib.sh / valu_attrib.py).
//                1 pre-test, 2 exchanged exact tests, 3 shading, 4 winner's hit record, 5 sincos.
//   PT_PROBE_EXTRA_LOAD      one more dwordx4 gather of a neighbouring pair record per inner
//                            traversal step, result kept live (tools/r03_probe.sh)
//   PT_PROBE_EXTRA_VALU=N    N dependent v_add_f32 per inner traversal step
//   PT_STAGE_REPS=N          k_bounce stages its LDS geom table N times per block (the price of
//                            the staging, results unchanged)
//   PT_SLEEP_WAVES=N         k_bounce waves PT_SLEEP_FROM..3 sleep N x 64 cycles after the staging
//   PT_EXTRA_ATOMIC          block_append waits for a second returning atomic (on the counter line's
//                            padding word) before releasing the block: the price of that latency
#ifndef PT_TOOL_HOOKS_H
#define PT_TOOL_HOOKS_H

#ifndef PT_DUP
#define PT_DUP 0
#endif

#define PT_HOOK(NAME, ...) PT_HOOK_##NAME(__VA_ARGS__)

#if PT_DUP == 1
#define PT_HOOK_DUP_CULL(sc, lg, ro, rd, bounded)                                              \
    do {                                                                                        \
        const f3 ro2_ = ro + mk(0.f, 0.f, 0.f);                                                 \
        const uint64_t c2_ = cull_candidates(sc, lg, cull_ray(ro2_, rd), ro2_, rd, bounded);    \
        asm volatile("" ::"v"((uint32_t)c2_), "v"((uint32_t)(c2_ >> 32)));                     \
    } while (0)
#else
#define PT_HOOK_DUP_CULL(...) ((void)0)
#endif

#if PT_DUP == 2
#define PT_HOOK_DUP_EXACT(geom, o, d)                                                           \
    do {                                                                                        \
        f3 s2_;                                                                                 \
        const float t2_ = geom_test(geom, o + mk(0.f, 0.f, 0.f), d, s2_);                       \
        asm volatile("" ::"v"(t2_), "v"(s2_.x), "v"(s2_.y), "v"(s2_.z));                      \
    } while (0)
#else
#define PT_HOOK_DUP_EXACT(...) ((void)0)
#endif

#if PT_DUP == 3
#define PT_HOOK_DUP_SHADE(TEX, sc, p, h, iter)                                                  \
    do {                                                                                        \
        PathReg q_ = p;                                                                         \
        q_.c = q_.c + mk(0.f, 0.f, 0.f);                                                        \
        shade_path<TEX>(sc, q_, h, iter + q_.slot, [&]() { return hit_attr(sc, h); });          \
        asm volatile("" ::"v"(q_.c.x), "v"(q_.c.y), "v"(q_.c.z), "v"(q_.d.x), "v"(q_.d.y),     \
                     "v"(q_.d.z), "v"(q_.o.x), "v"(q_.o.y), "v"(q_.o.z), "v"(q_.rb));            \
    } while (0)
#else
#define PT_HOOK_DUP_SHADE(...) ((void)0)
#endif

#if PT_DUP == 4
#define PT_HOOK_DUP_HIT(HAS_BVH, BVH_FAST, sc, o, d, stack, qt, qw, qs)                         \
    do {                                                                                        \
        const Hit h2_ = finish_hit<HAS_BVH, BVH_FAST>(sc, o, d + mk(0.f, 0.f, 0.f), stack, qt, qw, qs); \
        asm volatile("" ::"v"(h2_.t), "v"(h2_.n.x), "v"(h2_.n.y), "v"(h2_.n.z), "v"(h2_.mat)); \
    } while (0)
#else
#define PT_HOOK_DUP_HIT(...) ((void)0)
#endif

#if PT_DUP == 5
#define PT_HOOK_DUP_SINCOS(theta, xi)                                                           \
    do {                                                                                        \
        float s2_, c2_;                                                                         \
        pt_sincosf(theta + 0.0f * xi, &s2_, &c2_);                                              \
        asm volatile("" ::"v"(s2_), "v"(c2_));                                                 \
    } while (0)
#else
#define PT_HOOK_DUP_SINCOS(...) ((void)0)
#endif

#if defined(PT_PROBE_EXTRA_LOAD) || defined(PT_PROBE_EXTRA_VALU)
#ifndef PT_PROBE_EXTRA_VALU
#define PT_PROBE_EXTRA_VALU 0
#endif
#define PT_HOOK_PROBE_INNER(sc, cur, pr)                                                        \
    do {                                                                                        \
        if (PT_PROBE_LOAD_ON) {                                                                 \
            const v4f x_ = reinterpret_cast<const v4f*>(sc.pairs)[4 * (size_t)(cur ^ 1) + 1];   \
            asm volatile("" ::"v"(x_[0]));                                                      \
        }                                                                                       \
        float y_ = pr.l_lo.x;                                                                   \
        _Pragma("unroll") for (int k_ = 0; k_ < PT_PROBE_EXTRA_VALU; ++k_)                      \
            asm volatile("v_add_f32 %0, %0, %0" : "+v"(y_));                                    \
        asm volatile("" ::"v"(y_));                                                             \
    } while (0)
#ifdef PT_PROBE_EXTRA_LOAD
#define PT_PROBE_LOAD_ON 1
#else
#define PT_PROBE_LOAD_ON 0
#endif
#else
#define PT_HOOK_PROBE_INNER(...) ((void)0)
#endif

#if defined(PT_STAGE_REPS) && PT_STAGE_REPS > 1
#define PT_HOOK_STAGE_EXTRA(on, sc, s_dyn)                                                      \
    do {                                                                                        \
        if (on)                                                                                 \
            for (int r_ = 1; r_ < PT_STAGE_REPS; ++r_) {                                        \
                __syncthreads();                                                                \
                stage_geoms(sc, s_dyn);                                                         \
            }                                                                                   \
    } while (0)
#elif defined(PT_SLEEP_WAVES)
// PT_SLEEP_WAVES=N, PT_SLEEP_FROM=w: waves w..3 of every k_bounce block sleep N x 64 cycles after
// the staging (a stagger / delay probe, results unchanged)
#ifndef PT_SLEEP_FROM
#define PT_SLEEP_FROM 0
#endif
#define PT_HOOK_STAGE_EXTRA(on, sc, s_dyn)                                                      \
    do {                                                                                        \
        if ((threadIdx.x >> 6) >= PT_SLEEP_FROM)                                                \
            for (int r_ = 0; r_ < PT_SLEEP_WAVES; ++r_) __builtin_amdgcn_s_sleep(1);           \
    } while (0)
#else
#define PT_HOOK_STAGE_EXTRA(...) ((void)0)
#endif

#ifdef PT_EXTRA_ATOMIC
#define PT_HOOK_ATOMIC_EXTRA(sb, ctr)                                                           \
    do {                                                                                        \
        const int x_ = atomicAdd((ctr) + 1, 1);                                                 \
        int z_;                                                                                 \
        asm volatile("v_mov_b32 %0, 0" : "=v"(z_) : "v"(x_));                                   \
        (sb) += z_;                                                                             \
    } while (0)
#else
#define PT_HOOK_ATOMIC_EXTRA(...) ((void)0)
#endif

#endif  // PT_TOOL_HOOKS_H
