// hg_tune.hip -- variant launcher for tools/kbench.py (not part of the C ABI header;
// declared in include/sks_homography_tune.h).  Every variant computes the same bits
// as the shipped kernel; only the memory schedule differs.
#include <hip/hip_runtime.h>

#include "hg_aos.hpp"
#include "sks_homography.h"

namespace {

using namespace hg;

struct Variant {
    const char* name;
    int (*launch)(int algo, const float*, const float*, float*, int64_t, int, hipStream_t);
};

template <int P, int FL>
int launch_variant(int algo, const float* s, const float* t, float* H, int64_t n, int per_cu,
                   hipStream_t st) {
    const int64_t g = aos_grid<float, P, FL>(n, per_cu);
    if (algo == 0) solve_aos<kACA, true, float, P, FL><<<(unsigned)g, kBlock, 0, st>>>(s, t, H, n);
    else solve_aos<kSKS, true, float, P, FL><<<(unsigned)g, kBlock, 0, st>>>(s, t, H, n);
    return (int)hipGetLastError();
}

const Variant kVariants[] = {
    {"P4 nt-ld nt-st stage (shipped)", launch_variant<4, kNtLoad | kNtStore>},
    {"P4 plain", launch_variant<4, 0>},
    {"P4 nt-ld", launch_variant<4, kNtLoad>},
    {"P4 nt-st", launch_variant<4, kNtStore>},
    {"P8 nt-ld nt-st stage", launch_variant<8, kNtLoad | kNtStore>},
    {"P4 nt persist", launch_variant<4, kNtLoad | kNtStore | kPersist>},
    {"P4 nt lds-load", launch_variant<4, kNtLoad | kNtStore | kLdsLoad>},
    {"P8 nt lds-load", launch_variant<8, kNtLoad | kNtStore | kLdsLoad>},
    {"P4 nt direct-st", launch_variant<4, kNtLoad | kNtStore | kDirectSt>},
    {"P2 nt direct-st", launch_variant<2, kNtLoad | kNtStore | kDirectSt>},
    {"P1 nt direct-st", launch_variant<1, kNtLoad | kNtStore | kDirectSt>},
    {"P4 nt lds-load persist", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kPersist>},
    {"P4 plain lds-load", launch_variant<4, kLdsLoad>},
    {"P2 nt lds-load", launch_variant<2, kNtLoad | kNtStore | kLdsLoad>},
    {"P1 nt lds-load", launch_variant<1, kNtLoad | kNtStore | kLdsLoad>},
    {"P3 nt lds-load", launch_variant<3, kNtLoad | kNtStore | kLdsLoad>},
    {"P4 nt lds-dma", launch_variant<4, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P2 nt lds-dma", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma>},
    {"P4 lds-dma nt-st", launch_variant<4, kNtStore | kLdsLoad | kLdsDma>},
    {"P4 nt-ld lds-load plain-st", launch_variant<4, kNtLoad | kLdsLoad>},
    {"P2 nt stage", launch_variant<2, kNtLoad | kNtStore>},
    {"P2 nt lds-dma persist", launch_variant<2, kNtLoad | kNtStore | kLdsLoad | kLdsDma | kPersist>},
};

}  // namespace

extern "C" {

int hg_tune_num_variants(void) { return (int)(sizeof(kVariants) / sizeof(kVariants[0])); }

const char* hg_tune_variant_name(int v) {
    return (v >= 0 && v < hg_tune_num_variants()) ? kVariants[v].name : nullptr;
}

int hg_tune_aos_f32(int algo, int variant, const float* src, const float* tar, float* H,
                    int64_t n, int per_cu, void* stream) {
    if (variant < 0 || variant >= hg_tune_num_variants() || n <= 0 || (algo != 0 && algo != 1))
        return (int)hipErrorInvalidValue;
    return kVariants[variant].launch(algo, src, tar, H, n, per_cu > 0 ? per_cu : 8,
                                     reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
