// Build tag of one translation unit: which compile-time tuning / experiment defines it was built
// with.  Included FIRST by every source of libgeoflink_hip.so, after `#define GF_TU_NAME <name>`,
// so every GF_* macro seen here came from the compiler command line (the sources' own defaults
// are set later, under #ifndef).  gf_build_info() (api.cpp) concatenates the tags of all units;
// the smoke and the GPU suite require an empty list, so an experiment build cannot pass as the
// product.
//
// Experiment hooks (GF_*_EXP*) change results on purpose; they compile only together with
// GF_EXPERIMENT_BUILD, which tools/build_exp.sh adds and the Makefile's product rule never does.
#pragma once

#ifndef GF_TU_NAME
#error "define GF_TU_NAME before including gf_buildtag.hpp"
#endif

#define GF_BT_STR2(x) #x
#define GF_BT_STR(x) GF_BT_STR2(x)
#define GF_BT_CAT2(a, b) a##b
#define GF_BT_CAT(a, b) GF_BT_CAT2(a, b)

#if (defined(GF_RADIX_EXP) || defined(GF_RANGE_EXP) || defined(GF_SCAT_EXP_NOSTORE) ||          \
     defined(GF_BAND_EXP_NOSTAGE) || defined(GF_BAND_EXP_NOEMIT) || defined(GF_BAND_EXP_NOWALK) || \
     defined(GF_BAND_EXP_NOPUSH)) &&                                                             \
    !defined(GF_EXPERIMENT_BUILD)
#error "experiment hooks (GF_*_EXP*) need GF_EXPERIMENT_BUILD: build them with tools/build_exp.sh"
#endif

// one entry per knob: " NAME=value" when the command line set it, "" otherwise
#ifdef GF_EXPERIMENT_BUILD
#define GF_BT_IF_GF_EXPERIMENT_BUILD " GF_EXPERIMENT_BUILD"
#else
#define GF_BT_IF_GF_EXPERIMENT_BUILD ""
#endif
#ifdef GF_TRACE
#define GF_BT_IF_GF_TRACE " GF_TRACE"
#else
#define GF_BT_IF_GF_TRACE ""
#endif
#ifdef GF_RADIX_EXP
#define GF_BT_IF_GF_RADIX_EXP " GF_RADIX_EXP=" GF_BT_STR(GF_RADIX_EXP)
#else
#define GF_BT_IF_GF_RADIX_EXP ""
#endif
#ifdef GF_RANGE_EXP
#define GF_BT_IF_GF_RANGE_EXP " GF_RANGE_EXP=" GF_BT_STR(GF_RANGE_EXP)
#else
#define GF_BT_IF_GF_RANGE_EXP ""
#endif
#ifdef GF_SCAT_EXP_NOSTORE
#define GF_BT_IF_GF_SCAT_EXP_NOSTORE " GF_SCAT_EXP_NOSTORE"
#else
#define GF_BT_IF_GF_SCAT_EXP_NOSTORE ""
#endif
#if defined(GF_BAND_EXP_NOSTAGE) || defined(GF_BAND_EXP_NOEMIT) || defined(GF_BAND_EXP_NOWALK) || \
    defined(GF_BAND_EXP_NOPUSH)
#define GF_BT_IF_GF_BAND_EXP " GF_BAND_EXP_*"
#else
#define GF_BT_IF_GF_BAND_EXP ""
#endif
#ifdef GF_GEO_UNROLL
#define GF_BT_IF_GF_GEO_UNROLL " GF_GEO_UNROLL=" GF_BT_STR(GF_GEO_UNROLL)
#else
#define GF_BT_IF_GF_GEO_UNROLL ""
#endif
#ifdef GF_GEO_LINES
#define GF_BT_IF_GF_GEO_LINES " GF_GEO_LINES=" GF_BT_STR(GF_GEO_LINES)
#else
#define GF_BT_IF_GF_GEO_LINES ""
#endif
#ifdef GF_BUCKET_BITS
#define GF_BT_IF_GF_BUCKET_BITS " GF_BUCKET_BITS=" GF_BT_STR(GF_BUCKET_BITS)
#else
#define GF_BT_IF_GF_BUCKET_BITS ""
#endif
#ifdef GF_JOIN_BUCKET_U
#define GF_BT_IF_GF_JOIN_BUCKET_U " GF_JOIN_BUCKET_U=" GF_BT_STR(GF_JOIN_BUCKET_U)
#else
#define GF_BT_IF_GF_JOIN_BUCKET_U ""
#endif
#ifdef GF_BAND_BUF
#define GF_BT_IF_GF_BAND_BUF " GF_BAND_BUF=" GF_BT_STR(GF_BAND_BUF)
#else
#define GF_BT_IF_GF_BAND_BUF ""
#endif
#ifdef GF_BAND_R
#define GF_BT_IF_GF_BAND_R " GF_BAND_R=" GF_BT_STR(GF_BAND_R)
#else
#define GF_BT_IF_GF_BAND_R ""
#endif
#ifdef GF_BAND_R1
#define GF_BT_IF_GF_BAND_R1 " GF_BAND_R1=" GF_BT_STR(GF_BAND_R1)
#else
#define GF_BT_IF_GF_BAND_R1 ""
#endif
#ifdef GF_BAND_PAIR
#define GF_BT_IF_GF_BAND_PAIR " GF_BAND_PAIR=" GF_BT_STR(GF_BAND_PAIR)
#else
#define GF_BT_IF_GF_BAND_PAIR ""
#endif
#ifdef GF_BAND_FLATSEL
#define GF_BT_IF_GF_BAND_FLATSEL " GF_BAND_FLATSEL=" GF_BT_STR(GF_BAND_FLATSEL)
#else
#define GF_BT_IF_GF_BAND_FLATSEL ""
#endif
#ifdef GF_BAND_LDS_KB
#define GF_BT_IF_GF_BAND_LDS_KB " GF_BAND_LDS_KB=" GF_BT_STR(GF_BAND_LDS_KB)
#else
#define GF_BT_IF_GF_BAND_LDS_KB ""
#endif
#ifdef GF_BAND_THREADS
#define GF_BT_IF_GF_BAND_THREADS " GF_BAND_THREADS=" GF_BT_STR(GF_BAND_THREADS)
#else
#define GF_BT_IF_GF_BAND_THREADS ""
#endif
#ifdef GF_BAND_MINBLK
#define GF_BT_IF_GF_BAND_MINBLK " GF_BAND_MINBLK=" GF_BT_STR(GF_BAND_MINBLK)
#else
#define GF_BT_IF_GF_BAND_MINBLK ""
#endif
#ifdef GF_BAND_QUEUE
#define GF_BT_IF_GF_BAND_QUEUE " GF_BAND_QUEUE=" GF_BT_STR(GF_BAND_QUEUE)
#else
#define GF_BT_IF_GF_BAND_QUEUE ""
#endif
#ifdef GF_BAND_BALANCED
#define GF_BT_IF_GF_BAND_BALANCED " GF_BAND_BALANCED=" GF_BT_STR(GF_BAND_BALANCED)
#else
#define GF_BT_IF_GF_BAND_BALANCED ""
#endif
#ifdef GF_RANGE_WAVEQ
#define GF_BT_IF_GF_RANGE_WAVEQ " GF_RANGE_WAVEQ=" GF_BT_STR(GF_RANGE_WAVEQ)
#else
#define GF_BT_IF_GF_RANGE_WAVEQ ""
#endif
#ifdef GF_RANGE_VEC
#define GF_BT_IF_GF_RANGE_VEC " GF_RANGE_VEC=" GF_BT_STR(GF_RANGE_VEC)
#else
#define GF_BT_IF_GF_RANGE_VEC ""
#endif
#ifdef GF_RANGE_TEST_GROUP
#define GF_BT_IF_GF_RANGE_TEST_GROUP " GF_RANGE_TEST_GROUP=" GF_BT_STR(GF_RANGE_TEST_GROUP)
#else
#define GF_BT_IF_GF_RANGE_TEST_GROUP ""
#endif
#ifdef GF_RANGE_WAVES
#define GF_BT_IF_GF_RANGE_WAVES " GF_RANGE_WAVES=" GF_BT_STR(GF_RANGE_WAVES)
#else
#define GF_BT_IF_GF_RANGE_WAVES ""
#endif
#ifdef GF_RANGE_U
#define GF_BT_IF_GF_RANGE_U " GF_RANGE_U=" GF_BT_STR(GF_RANGE_U)
#else
#define GF_BT_IF_GF_RANGE_U ""
#endif

namespace gf {
// " NAME=value ..." of this unit's command-line knobs; "" for a product build
const char* GF_BT_CAT(build_tag_, GF_TU_NAME)() {
  return GF_BT_IF_GF_EXPERIMENT_BUILD GF_BT_IF_GF_TRACE GF_BT_IF_GF_RADIX_EXP GF_BT_IF_GF_RANGE_EXP
      GF_BT_IF_GF_SCAT_EXP_NOSTORE GF_BT_IF_GF_BAND_EXP GF_BT_IF_GF_GEO_UNROLL GF_BT_IF_GF_GEO_LINES
          GF_BT_IF_GF_BUCKET_BITS GF_BT_IF_GF_JOIN_BUCKET_U GF_BT_IF_GF_BAND_BUF GF_BT_IF_GF_BAND_R
              GF_BT_IF_GF_BAND_R1 GF_BT_IF_GF_BAND_PAIR GF_BT_IF_GF_BAND_FLATSEL GF_BT_IF_GF_BAND_LDS_KB
                  GF_BT_IF_GF_BAND_MINBLK GF_BT_IF_GF_BAND_THREADS GF_BT_IF_GF_BAND_QUEUE GF_BT_IF_GF_BAND_BALANCED
                      GF_BT_IF_GF_RANGE_WAVEQ GF_BT_IF_GF_RANGE_VEC GF_BT_IF_GF_RANGE_TEST_GROUP
                          GF_BT_IF_GF_RANGE_WAVES GF_BT_IF_GF_RANGE_U;
}
}  // namespace gf
