// spe.hip -- MI355X (gfx950) shortest-path engine for Shadow's topology routing.
//
// Replaces, for every attached (source, target) pair at once, what the
// reference computes lazily per cache miss in src/main/routing/shd-topology.c:
//   DIRECT  _topology_lookupDirectPath           :1862-1912
//   SSSP    _topology_computeSourcePaths          :1640-1860 (igraph Dijkstra :1741)
//           + _topology_computePathProperties     :1392-1508
//   SELF    _topology_computeShortestPathToSelf   :1530-1638
// and serves the per-packet queries (topology_getLatency/getReliability/
// isRoutable, :2048-2075) from an HBM-resident table.
//
// Kernels (all hand-written for CDNA4, wave64):
//   k_init_state   per-batch state reset (dist = +inf, parent = none)
//   k_seed         sources -> first frontier marks
//   k_relax        multi-source label-correcting relaxation over a dense
//                  frontier bitmap (wave-ballot compaction, no global counter):
//                  ONE WAVE = one vertex x 64 sources (lane = source).  Only
//                  in-neighbours that changed last round are read (their flags
//                  are ballot-scanned 64 at a time; 4 coalesced 512-B rows of the
//                  [vertex][64] state); the canonical parent (alt, dist[u], u)
//                  and the path-order reliability / hop count / first hop are
//                  carried with the distance, so converged state IS the row.
//   k_rows_sssp    state -> table rows (+ SELF / [s] rules, slow path-walk for
//                  targets with vertex loss or multigraph get_eid latencies)
//   k_rows_direct  complete graphs: every pair is the direct edge
//   k_direct_overlay  preferdirectpaths: adjacent pairs get the direct edge
//   k_sssp_lds     small graphs (<= 10,240 relaxation vertices): one workgroup per
//                  source row, relaxation state in LDS, rows written directly
//   k_owner_replay compat: the reference's first-writer-wins path cache
//   k_lookup       batched per-packet (s, t) -> (latency, reliability, ok)
//   k_min_latency  minimumPathLatency reduction
// plus the host side: graph upload, table build loop, on-disk table cache.
//
// One translation unit in parts (shadow_amd/csrc/spe/): kernels_relax.inc,
// kernels_rows.inc, kernels_lds.inc, kernels_fw.inc (inside this file's anonymous
// namespace), then host_graph.inc, host_table.inc, host_build.inc, host_api.inc.
//
// Bit-exactness: every distance is the least fixpoint of
// d[v] = min_u fl(d[u] + w), which igraph's Dijkstra also computes (IEEE
// round-to-nearest addition is monotone); compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <random>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "spe_internal.h"

#define WAVE 64
#define BLOCK 256

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define ABI_MSG(T) (std::string(T) + ".struct_size is not sizeof(" T ") of this libspe: the caller was built " \
                    "against another include/spe.h (set it with SPE_STRUCT_INIT)")

// FNV-1a 64 over raw bytes (table cache keys)
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) {
            h ^= b[i];
            h *= 1099511628211ull;
        }
    }
    template <typename T>
    void val(const T& x) { add(&x, sizeof(x)); }
};

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(SPE_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

constexpr double INF = __builtin_inf();

struct DevGraph {
    int32_t n;               // relaxation vertices (the core when pendants are pruned)
    int32_t nrel;
    int32_t n_full;          // all vertices (original ids)
    const int32_t* iptr;
    const int32_t* icol;
    const int4* ipack;       // per in-entry, one 16-B load for the relaxation: {icol, orev | heavy[icol] << 31
                             // (undirected: the out-list is the in-list), iw as two 32-bit halves}
    const int32_t* irow;     // in-CSR entry -> its target vertex (flat edge passes)
    const uint32_t* ipair;   // nc <= 65535 only (LDS-engine graphs): (irow << 16) | icol, one 4-B load
    const double* iw;
    const double* ia;
    const double* iwrep;
    const int32_t* optr;
    const int32_t* ocol;
    const int32_t* orev;     // out-entry -> index of the same edge in the target's in-CSR list
    const double* owrep;
    const double* oarep;
    const double* ow;        // relaxation (lightest) weight per out-entry (== iw when undirected)
    int32_t undirected;      // out-CSR == in-CSR
    const uint8_t* heavy;    // [n] in-degree > 64
    const uint8_t* oheavy;   // [out entry] heavy[target]: which frontier buffer it goes to
    int32_t ablate;          // diagnostic only (SPE_ABLATE env): bit 0 = skip route records
    const double* vfac;
    const double* loop_w;
    const double* loop_a;
    const double* self_w2;
    const double* self_a2;
    const int32_t* self_other;
    // original <-> relaxation ids and the full in-CSR (pendant edges, DIRECT lookups)
    const int32_t* core_id;      // [n_full] -1 = pruned pendant
    const int32_t* corev;        // [n]
    const int32_t* anchor_core;  // [n_full]
    const int32_t* fiptr;
    const double* fiw;
    const double* fia;
    const double* fiwrep;
    // optional per-edge auxiliary attribute of the get_eid edge (spe_graph_set_edge_aux)
    const double* iaux;          // [relaxation in-CSR entry]
    const double* fiaux;         // [full in-CSR entry]
    const int32_t* dptr;         // DIRECT lookups: full out-CSR
    const int32_t* dcol;
    const double* dwrep;
    const double* darep;
    // Degree-3 contraction (spe_graph.devx, the batch engine's graph when the
    // table runs on it; NULL in the plain graph).  Relaxation ids are then the kept
    // vertices; entry k offers fl(fl(d[icol[k]] + iw[k]) + xw2[k]) (xw2 = 0 for a plain
    // edge: the same bits as one add), its parent of record is core vertex xkey[k] (x
    // for a shortcut), and the route multiplies ia[k] then xa2[k] and adds 1 + (xvia >= 0)
    // hops.  A removed vertex's rows come from its three neighbours (rnb / rw / ra).
    const double* xw2;
    const double* xa2;
    const int32_t* xkey;
    const int32_t* xvia;         // original id of x, -1 for a plain edge
    const int32_t* xrm;          // [n_full] removed index, -1 otherwise
    const int32_t* rnb;          // [3 removed] kept ids of the neighbours (increasing)
    const double* rw;
    const double* ra;
};

struct RowMode {
    int32_t complete;
    int32_t prefer;
    int32_t self_mode;
    int32_t multi_rep;
    int32_t directed;
};

// Per-lane route record carried with the distance: the path-order reliability
// fold (starting at the source factor) and (hops, first hop).  16 B so a parent
// lookup is ONE 16-B access per lane (lanes with the same parent coalesce).
struct alignas(16) Route {
    double r;
    int32_t h;
    int32_t f;
};

// Relaxation state of one batch, [lane group][vertex][L lanes] (lane = source).
// A lane group of L sources is the unit that shares a frontier; a wave holds
// 64/L subgroups and so relaxes 64/L (group, vertex) items at once.
struct State {
    double* D;        // distance
    int32_t* P;       // in-CSR index of the chosen parent edge, -1 none
    Route* RT;        // route record
};

typedef double dvec2 __attribute__((ext_vector_type(2)));

struct Table {
    double2* lr;      // {latency, reliability}: one 16-B record, so a lookup is one HBM line
    int32_t* next;
    uint16_t* hops;
    int32_t A;
    int32_t* prev;    // owner-replay mode only: vertex before the target on the path
    double* aux;      // want_aux only: path-order sum of the edges' auxiliary attribute
};

__device__ __forceinline__ bool has_attr(double x) { return !__builtin_isnan(x); }

__device__ __forceinline__ size_t tidx(int32_t sb_local, int32_t A, int32_t j, int32_t lane) {
    return ((size_t)sb_local * (size_t)A + (size_t)j) * WAVE + (size_t)lane;
}

template <int L>
struct Sub {
    static constexpr int V = WAVE / L;                                   // subgroups per wave
    static constexpr uint64_t MASK = (L == 64) ? ~0ull : ((1ull << L) - 1);
    static constexpr int INFL = (L == 64) ? 8 : (L == 32 ? 6 : 4);       // neighbour rows in flight per subgroup
};

template <int L>
__device__ __forceinline__ size_t sidx(int32_t g, int32_t n, int32_t v, int32_t j) {
    return ((size_t)g * (size_t)n + (size_t)v) * L + (size_t)j;
}

// value of `x` held by lane `src` (same subgroup, active)
template <int L>
__device__ __forceinline__ int32_t sub_get(int32_t x, int32_t src) {
    if constexpr (L == 64) return __builtin_amdgcn_readlane(x, src);
    else return __shfl(x, src);
}

template <int L>
__device__ __forceinline__ double sub_get_d(double x, int32_t src) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)sub_get<L>((int32_t)(uint32_t)b, src);
    const uint32_t hi = (uint32_t)sub_get<L>((int32_t)(uint32_t)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

#include "spe/kernels_relax.inc"
#include "spe/kernels_rows.inc"
#include "spe/kernels_lds.inc"
#include "spe/kernels_fw.inc"
}  // namespace

#include "spe/host_graph.inc"
#include "spe/host_table.inc"
#include "spe/host_build.inc"
#include "spe/host_api.inc"
