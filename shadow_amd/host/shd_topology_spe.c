/*
 * shd_topology_spe.c -- the reference's topology API (src/main/routing/
 * shd-topology.{c,h}) re-hosted on the MI355X path engine (include/spe.h).
 *
 * What stays on the host (C, as in the reference):
 *   GraphML ingest + validation       shd-topology.c:356-384, 550-1195
 *   host attachment by hints / LPM    shd-topology.c:2077-2413
 *   IP -> vertex map, packet counters shd-topology.c:1373-1390, shd-path.c:53-56
 * What moves to the GPU (spe_table_build, once, at the first query):
 *   every (source, target) row the reference computed lazily per cache miss
 *   with igraph Dijkstra under the global graphLock (shd-topology.c:1640-1912).
 * Queries are then lock-free reads of the sealed table's host mirror.
 *
 * Semantics differences, all documented in DESIGN.md:
 *   - per-source rows: (s,t) is always tree_s(s->t).  The reference returns
 *     whichever of tree_s(s->t) / tree_t(t->s) was cached first (first-writer
 *     wins, shd-topology.c:1292-1321) -- identical values whenever both rows
 *     agree, which is every DIRECT pair and every undirected pair whose
 *     forward/backward sums round the same.
 *   - (s,s) uses the row's [s] path when s has a self-loop (SPE_SELF_ROW).
 */
#include "shd_topology_spe.h"

#include <arpa/inet.h>
#include <math.h>
#include <netinet/in.h>
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <libxml/parser.h>
#include <libxml/tree.h>

#include "spe.h"

#ifdef SHD_TOPOLOGY_SPE_PREFIXED   /* the header declared spe_topology_*: define those */
#define topology_attach spe_topology_attach
#define topology_attached_vertex spe_topology_attached_vertex
#define topology_cached_path_count spe_topology_cached_path_count
#define topology_check_graphml spe_topology_check_graphml
#define topology_detach spe_topology_detach
#define topology_free spe_topology_free
#define topology_getLatency spe_topology_getLatency
#define topology_getPathInfo spe_topology_getPathInfo
#define topology_getPathInfoBatch spe_topology_getPathInfoBatch
#define topology_incrementPathPacketCounterBatch spe_topology_incrementPathPacketCounterBatch
#define topology_getReliability spe_topology_getReliability
#define topology_incrementPathPacketCounter spe_topology_incrementPathPacketCounter
#define topology_isRoutable spe_topology_isRoutable
#define topology_min_path_latency spe_topology_min_path_latency
#define topology_new spe_topology_new
#define topology_new_on_device spe_topology_new_on_device
#define topology_path_packet_count spe_topology_path_packet_count
#define topology_seal spe_topology_seal
#define topology_set_answer_mode spe_topology_set_answer_mode
#define topology_set_log_callback spe_topology_set_log_callback
#define topology_set_log_level spe_topology_set_log_level
#define topology_set_min_latency_callback spe_topology_set_min_latency_callback
#define topology_vertex_count spe_topology_vertex_count
#endif

enum { LOG_ERROR = 0, LOG_CRITICAL, LOG_WARNING, LOG_MESSAGE, LOG_INFO, LOG_DEBUG };

/* vertex string / numeric attributes the reference reads, by exact name */
enum { VS_ID = 0, VS_IP, VS_CITYCODE, VS_COUNTRYCODE, VS_GEOCODE, VS_TYPE, VS_COUNT };
enum { VN_BWDOWN = 0, VN_BWUP, VN_PACKETLOSS, VN_ASN, VN_COUNT };
static const char* VS_NAMES[VS_COUNT] = {"id", "ip", "citycode", "countrycode", "geocode", "type"};
static const char* VN_NAMES[VN_COUNT] = {"bandwidthdown", "bandwidthup", "packetloss", "asn"};

/* One record of the path-cache model per ORDERED vertex pair (x, y) that has an
 * explicitly stored Path (a DIRECT or SELF store) or a packet count.  Rows stored
 * by a source's Dijkstra run are implicit (run_seq); see "path cache model". */
enum { K_NONE = 0, K_DIRECT, K_SELF };
typedef struct {
    uint64_t key;      /* ((uint64_t)x << 32 | y) + 1, 0 = empty */
    uint64_t seq;      /* store sequence of an explicit entry, 0 = none */
    uint64_t count;    /* Path.packetCount (shd-path.c:53-56) of entry (x, y) */
    int32_t kind;      /* K_DIRECT / K_SELF when seq > 0 */
} PairRec;

/* one slot of the address map: v >= 0 the vertex, IP_EMPTY / IP_GONE (a detached address) */
enum { IP_EMPTY = -1, IP_GONE = -2 };
typedef struct {
    uint32_t ip;
    int32_t v;
} IpSlot;

#define NSHARD 64
typedef struct {
    pthread_mutex_t mu;
    PairRec* tab;
    size_t cap, size;
} Shard;

/* The state lock, sharded by reader: each thread takes its own slot's rwlock shared
 * (its reader count on a cache line of its own), attach / detach / publish take every
 * slot exclusive in slot order.  One shared rwlock bounced its reader count between
 * the workers' cores on every call: 16 threads of single calls on the host-mirrored
 * C3 table ran 4.8M calls/s in all against 4.0M/s on one thread.  Each slot prefers
 * writers: a table swap or an attach must not starve behind a steady stream of
 * queries (glibc's default prefers readers). */
#define STATE_SLOTS 32
typedef struct {
    pthread_rwlock_t l;
    char pad[128 - sizeof(pthread_rwlock_t)];
} StateSlot;

static _Atomic int state_slot_next;
static _Thread_local int state_slot = -1;

static int my_state_slot(void) {
    if (state_slot < 0) state_slot = atomic_fetch_add(&state_slot_next, 1) % STATE_SLOTS;
    return state_slot;
}

/* An immutable sealed table: published under the state lock, replaced whole (never
 * modified) when hosts attach after sealing, and freed only after the writer
 * lock has drained every reader that could hold it. */
typedef struct {
    int32_t A;
    int32_t* slot_of_vertex;       /* [n] slot, -1 = not in this table */
    int32_t* attached;             /* [A] slot -> vertex */
    spe_table* table;
    double* mlat;                  /* full host mirror [A][A], or NULL */
    double* mrel;
    _Atomic(double*)* blocks;      /* lazy mirror per SOURCE ROW: lat[A], rel[A] (a row is 16 A bytes:
                                    * 1.6 MB at A = 100k, where a 64-source block was 102 MB) */
    _Atomic uint8_t* touch;        /* single reads of each row so far (a row is mirrored on its
                                    * ROW_MIRROR_AFTER-th: a row read a few times is cheaper as
                                    * single records) */
    _Atomic int64_t row_budget;    /* bytes left for lazy rows; beyond it: spe_table_get_latrel */
    _Atomic int host_reads;        /* spe_table_layout.host_reads of the table (-1: not known yet) */
    int64_t mirror_budget;         /* the budget this snapshot was given (full or lazy) */
    pthread_mutex_t row_mu;
    double min_latency;            /* over every routable entry */
} Snap;

struct _Topology {
    int32_t device;
    int32_t n;
    int64_t m;
    int32_t directed;
    int32_t prefer_direct;
    int32_t complete;
    int32_t shared_rows_exact;     /* spe_graph_info.shared_rows_exact: shared / derived rows are bit-exact */
    /* graph, edge list form (GraphML order) */
    int32_t *esrc, *edst;
    double *elat, *eloss;
    char** vstr[VS_COUNT];     /* NULL array = attribute absent from the graph */
    uint32_t* vip;             /* [n] address_stringToIP of each vertex's "ip" (INADDR_NONE when absent) */
    uint64_t* vip_index;       /* (ip << 32 | v) of every vertex with a usable ip, sorted: exact hints in O(log n) */
    int64_t n_vip;
    double* vnum[VN_COUNT];
    spe_graph* graph;

    /* the state lock (state_rdlock / state_wrlock) guards the IP map, the attached set
     * and the published snapshot; queries hold it shared for their whole duration,
     * attach / publish exclusive */
    StateSlot* state;
    IpSlot* ips;               /* open-addressed address -> vertex map: one 8-B slot per probe */
    size_t ip_cap, ip_size;
    uint8_t* is_attached;      /* [n] */
    int32_t* attached;         /* vertices in first-attach order */
    int32_t n_attached;
    Snap* snap;

    pthread_mutex_t seal_lock; /* one table build at a time */
    double build_seconds;
    int64_t build_rows;

    /* path cache model (shd-topology.c:1269-1371, 1952-2034): run_seq[v] = store
     * sequence of v's first Dijkstra row run; explicit entries and packet counts
     * in sharded maps; cache_mu serialises misses (the reference's store path) */
    pthread_mutex_t cache_mu;
    pthread_mutex_t batch_mu;  /* the cached batch scratch below (one batch at a time uses it) */
    void* bscr;
    size_t bscr_bytes;
    _Atomic uint64_t* run_seq;
    _Atomic uint8_t* xflag;    /* [n] 1: some explicit entry (x, .) exists -- readers skip the
                                  shard (and its mutex) for every other x */
    _Atomic uint64_t seq;
    _Atomic int64_t n_explicit;
    Shard shards[NSHARD];
    int32_t cache_mode;        /* TOPOLOGY_ANSWER_ROWS | TOPOLOGY_ANSWER_REFERENCE */
    _Atomic uint64_t stored_min_bits;   /* minimumPathLatency over stored entries (reference mode) */
    int64_t self_paths;

    int32_t log_level;
    topology_log_fn log_fn;
    void* log_ctx;
    topology_min_latency_fn minlat_fn;
    void* minlat_ctx;
};

static void state_init(Topology* top) {
    top->state = aligned_alloc(128, STATE_SLOTS * sizeof(StateSlot));
    pthread_rwlockattr_t ra;
    pthread_rwlockattr_init(&ra);
    pthread_rwlockattr_setkind_np(&ra, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
    for (int i = 0; i < STATE_SLOTS; ++i) pthread_rwlock_init(&top->state[i].l, &ra);
    pthread_rwlockattr_destroy(&ra);
}

static void state_destroy(Topology* top) {
    if (!top->state) return;
    for (int i = 0; i < STATE_SLOTS; ++i) pthread_rwlock_destroy(&top->state[i].l);
    free(top->state);
    top->state = NULL;
}

static void state_rdlock(const Topology* top) { pthread_rwlock_rdlock(&top->state[my_state_slot()].l); }
static void state_rdunlock(const Topology* top) { pthread_rwlock_unlock(&top->state[my_state_slot()].l); }

static void state_wrlock(Topology* top) {
    for (int i = 0; i < STATE_SLOTS; ++i) pthread_rwlock_wrlock(&top->state[i].l);
}

static void state_wrunlock(Topology* top) {
    for (int i = STATE_SLOTS - 1; i >= 0; --i) pthread_rwlock_unlock(&top->state[i].l);
}

static int log_on(const Topology* top, int level) { return !top || level <= top->log_level; }

static void tlog(Topology* top, int level, const char* fmt, ...) {
    if (!log_on(top, level)) return;
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (top && top->log_fn) top->log_fn(level, buf, top->log_ctx);
    else if (level <= LOG_WARNING) fprintf(stderr, "[shd-topology-spe] %s\n", buf);
}

/* ------------------------------------------------------------ GraphML */

/* igraph attribute types of the GraphML reader: int/long/float/double -> numeric,
 * boolean -> boolean, string (or no attr.type) -> string */
enum { AT_STRING = 0, AT_NUMERIC, AT_BOOLEAN };

typedef struct {
    char* id;
    char* name;
    int numeric;   /* attr.type int/long/float/double */
    int atype;     /* AT_* */
    int for_;      /* 0 graph, 1 node, 2 edge, 3 all */
    char* def;
} GKey;

/* _topology_is{Graph,Vertex,Edge}AttributeKey (shd-topology.c:178-181, 235-238,
 * 264-267): g_ascii_strncasecmp over the canonical name's length, i.e. the
 * attribute name starts with the canonical one, case-insensitively */
static int attr_prefix(const char* name, const char* canonical) {
    return name && !strncasecmp(name, canonical, strlen(canonical));
}

static int key_in(const GKey* k, int domain) { return k->for_ == domain || k->for_ == 3; }

static int has_exact(const GKey* keys, size_t nkeys, int domain, const char* name) {
    for (size_t i = 0; i < nkeys; ++i)
        if (key_in(&keys[i], domain) && keys[i].name && !strcmp(keys[i].name, name)) return 1;
    return 0;
}

/* _topology_checkGraphAttributes, shd-topology.c:550-707.  Attributes are listed
 * per domain in declaration order (igraph_cattribute_list).  Each one whose name
 * prefix-matches a known attribute gets a type check whose result OVERWRITES
 * isSuccess (:588, :605-623, :666-670) instead of AND-ing into it; the
 * required-attribute checks (exact igraph names, :635-659, :675-690) can only
 * clear it.  So a type error is forgiven when a later checked attribute passes,
 * and only the last prefix-matched edge attribute's type counts in the end. */
static int check_attribute_types(Topology* top, const GKey* keys, size_t nkeys);

static const struct {
    const char* name;
    int type;
} VCHECK[] = {{"id", AT_STRING},          {"ip", AT_STRING},        {"citycode", AT_STRING},
              {"countrycode", AT_STRING}, {"asn", AT_NUMERIC},      {"type", AT_STRING},
              {"bandwidthdown", AT_NUMERIC}, {"bandwidthup", AT_NUMERIC}, {"packetloss", AT_NUMERIC},
              {"geocode", AT_STRING}},
  ECHECK[] = {{"latency", AT_NUMERIC}, {"jitter", AT_NUMERIC}, {"packetloss", AT_NUMERIC}};

static int type_ok(Topology* top, const GKey* k, int want) {   /* _topology_checkAttributeType */
    if (k->atype == want) return 1;
    tlog(top, LOG_WARNING, "attribute '%s' has an unexpected type (expected %s)", k->name,
         want == AT_NUMERIC ? "NUMERIC" : "STRING");
    return 0;
}

static int check_attribute_types(Topology* top, const GKey* keys, size_t nkeys) {
    int isSuccess = 1;
    for (size_t i = 0; i < nkeys; ++i) {   /* graph attributes */
        if (!key_in(&keys[i], 0) || !keys[i].name) continue;
        if (attr_prefix(keys[i].name, "preferdirectpaths")) isSuccess = type_ok(top, &keys[i], AT_STRING);
        else tlog(top, LOG_WARNING, "graph attribute '%s' is unsupported and will be ignored", keys[i].name);
    }
    for (size_t i = 0; i < nkeys; ++i) {   /* vertex attributes: first matching name, in the reference's order */
        if (!key_in(&keys[i], 1) || !keys[i].name) continue;
        size_t a = 0;
        while (a < sizeof VCHECK / sizeof VCHECK[0] && !attr_prefix(keys[i].name, VCHECK[a].name)) ++a;
        if (a < sizeof VCHECK / sizeof VCHECK[0]) isSuccess = type_ok(top, &keys[i], VCHECK[a].type);
        else tlog(top, LOG_INFO, "vertex attribute '%s' is unsupported and will be ignored", keys[i].name);
    }
    /* required vertex attributes ("id" is always defined: igraph stores the node ids) */
    if (!has_exact(keys, nkeys, 1, "bandwidthdown") || !has_exact(keys, nkeys, 1, "bandwidthup")) {
        tlog(top, LOG_WARNING, "the vertex attributes 'bandwidthdown' and 'bandwidthup' of type 'NUMERIC' are "
                               "required but not provided");
        isSuccess = 0;
    }
    for (size_t i = 0; i < nkeys; ++i) {   /* edge attributes */
        if (!key_in(&keys[i], 2) || !keys[i].name) continue;
        size_t a = 0;
        while (a < sizeof ECHECK / sizeof ECHECK[0] && !attr_prefix(keys[i].name, ECHECK[a].name)) ++a;
        if (a < sizeof ECHECK / sizeof ECHECK[0]) isSuccess = type_ok(top, &keys[i], ECHECK[a].type);
        else tlog(top, LOG_INFO, "edge attribute '%s' is unsupported and will be ignored", keys[i].name);
    }
    if (!has_exact(keys, nkeys, 2, "latency") || !has_exact(keys, nkeys, 2, "packetloss")) {
        tlog(top, LOG_WARNING, "the edge attributes 'latency' and 'packetloss' of type 'NUMERIC' are required but "
                               "not provided");
        isSuccess = 0;
    }
    if (isSuccess) tlog(top, LOG_MESSAGE, "successfully verified all graph, vertex, and edge attributes");
    else tlog(top, LOG_WARNING, "we could not properly validate all graph, vertex, and edge attributes");
    return isSuccess;
}

static char* xstrdup(const xmlChar* s) { return s ? strdup((const char*)s) : NULL; }

static double parse_num(const char* s) {
    if (!s) return NAN;
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') s++;
    if (*s == '\0') return NAN;
    return strtod(s, NULL);
}

static int key_for(const char* f) {
    if (!f || !strcmp(f, "all")) return 3;
    if (!strcmp(f, "graph")) return 0;
    if (!strcmp(f, "node")) return 1;
    if (!strcmp(f, "edge")) return 2;
    return 3;
}

/* vertex index = order of first reference (igraph's GraphML id trie) */
typedef struct {
    char** names;
    size_t n, cap;
    char** hkeys;
    int32_t* hvals;
    size_t hcap;
} NameMap;

static uint64_t hash_str(const char* s) {
    uint64_t h = 1469598103934665603ull;
    for (; *s; ++s) h = (h ^ (uint8_t)*s) * 1099511628211ull;
    return h;
}

static int32_t name_index(NameMap* nm, const char* name) {
    if (nm->n * 2 + 2 > nm->hcap) {
        size_t nc = nm->hcap ? nm->hcap * 2 : 1024;
        char** nk = calloc(nc, sizeof(char*));
        int32_t* nv = calloc(nc, sizeof(int32_t));
        for (size_t i = 0; i < nm->hcap; ++i)
            if (nm->hkeys[i]) {
                size_t j = hash_str(nm->hkeys[i]) & (nc - 1);
                while (nk[j]) j = (j + 1) & (nc - 1);
                nk[j] = nm->hkeys[i];
                nv[j] = nm->hvals[i];
            }
        free(nm->hkeys);
        free(nm->hvals);
        nm->hkeys = nk;
        nm->hvals = nv;
        nm->hcap = nc;
    }
    size_t j = hash_str(name) & (nm->hcap - 1);
    while (nm->hkeys[j]) {
        if (!strcmp(nm->hkeys[j], name)) return nm->hvals[j];
        j = (j + 1) & (nm->hcap - 1);
    }
    if (nm->n == nm->cap) {
        nm->cap = nm->cap ? nm->cap * 2 : 1024;
        nm->names = realloc(nm->names, nm->cap * sizeof(char*));
    }
    char* copy = strdup(name);
    nm->names[nm->n] = copy;
    nm->hkeys[j] = copy;
    nm->hvals[j] = (int32_t)nm->n;
    return (int32_t)nm->n++;
}

typedef struct {
    int32_t v;
    xmlNode* el;
} NodeRef;

static int load_graphml(Topology* top, const char* path) {
    xmlDoc* doc = xmlReadFile(path, NULL, XML_PARSE_NONET | XML_PARSE_HUGE | XML_PARSE_NOBLANKS);
    if (!doc) {
        tlog(top, LOG_CRITICAL, "unable to parse graphml file '%s'", path);
        return 0;
    }
    xmlNode* root = xmlDocGetRootElement(doc);
    GKey* keys = NULL;
    size_t nkeys = 0, capkeys = 0;
    xmlNode* graph = NULL;
    for (xmlNode* c = root ? root->children : NULL; c; c = c->next) {
        if (c->type != XML_ELEMENT_NODE) continue;
        if (!xmlStrcmp(c->name, (const xmlChar*)"key")) {
            if (nkeys == capkeys) {
                capkeys = capkeys ? capkeys * 2 : 16;
                keys = realloc(keys, capkeys * sizeof(GKey));
            }
            GKey* k = &keys[nkeys++];
            memset(k, 0, sizeof *k);
            xmlChar* a = xmlGetProp(c, (const xmlChar*)"id");
            k->id = xstrdup(a);
            xmlFree(a);
            a = xmlGetProp(c, (const xmlChar*)"attr.name");
            k->name = xstrdup(a);
            xmlFree(a);
            a = xmlGetProp(c, (const xmlChar*)"attr.type");
            k->numeric = a && (!xmlStrcmp(a, (const xmlChar*)"int") || !xmlStrcmp(a, (const xmlChar*)"long") ||
                               !xmlStrcmp(a, (const xmlChar*)"float") || !xmlStrcmp(a, (const xmlChar*)"double"));
            k->atype = k->numeric ? AT_NUMERIC
                                  : (a && !xmlStrcmp(a, (const xmlChar*)"boolean") ? AT_BOOLEAN : AT_STRING);
            xmlFree(a);
            a = xmlGetProp(c, (const xmlChar*)"for");
            k->for_ = key_for((const char*)a);
            xmlFree(a);
            for (xmlNode* d = c->children; d; d = d->next)
                if (d->type == XML_ELEMENT_NODE && !xmlStrcmp(d->name, (const xmlChar*)"default")) {
                    xmlChar* t = xmlNodeGetContent(d);
                    k->def = xstrdup(t);
                    xmlFree(t);
                }
        } else if (!xmlStrcmp(c->name, (const xmlChar*)"graph") && !graph) {
            graph = c;
        }
    }
    int ok = 1;
    if (!graph) {
        tlog(top, LOG_CRITICAL, "graphml file '%s' has no <graph>", path);
        ok = 0;
        goto out;
    }
    {
        xmlChar* ed = xmlGetProp(graph, (const xmlChar*)"edgedefault");
        top->directed = !(ed && !xmlStrcmp(ed, (const xmlChar*)"undirected"));
        xmlFree(ed);
    }
    /* first pass: vertex ids, edge count, graph data */
    NameMap nm;
    memset(&nm, 0, sizeof nm);
    size_t ne = 0, ncap = 0;
    NodeRef* nodes = NULL;
    size_t nn = 0;
    const char* pref_val = NULL;
    char* pref_key = NULL;
    for (size_t i = 0; i < nkeys; ++i)
        if (keys[i].name && (keys[i].for_ == 0 || keys[i].for_ == 3) && !strcmp(keys[i].name, "preferdirectpaths"))
            pref_key = keys[i].id;
    xmlChar* pref_text = NULL;
    for (xmlNode* c = graph->children; c; c = c->next) {
        if (c->type != XML_ELEMENT_NODE) continue;
        if (!xmlStrcmp(c->name, (const xmlChar*)"node")) {
            xmlChar* id = xmlGetProp(c, (const xmlChar*)"id");
            int32_t v = name_index(&nm, id ? (const char*)id : "");
            xmlFree(id);
            if (nn == ncap) {
                ncap = ncap ? ncap * 2 : 1024;
                nodes = realloc(nodes, ncap * sizeof(NodeRef));
            }
            nodes[nn].v = v;
            nodes[nn].el = c;
            nn++;
        } else if (!xmlStrcmp(c->name, (const xmlChar*)"edge")) {
            xmlChar* s = xmlGetProp(c, (const xmlChar*)"source");
            xmlChar* t = xmlGetProp(c, (const xmlChar*)"target");
            name_index(&nm, s ? (const char*)s : "");
            name_index(&nm, t ? (const char*)t : "");
            xmlFree(s);
            xmlFree(t);
            ne++;
        } else if (!xmlStrcmp(c->name, (const xmlChar*)"data") && pref_key) {
            xmlChar* k = xmlGetProp(c, (const xmlChar*)"key");
            if (k && !strcmp((const char*)k, pref_key)) {
                if (pref_text) xmlFree(pref_text);
                pref_text = xmlNodeGetContent(c);
            }
            xmlFree(k);
        }
    }
    if (pref_text) pref_val = (const char*)pref_text;
    else if (pref_key)
        for (size_t i = 0; i < nkeys; ++i)
            if (keys[i].id == pref_key) pref_val = keys[i].def;
    /* preferdirectpaths: string, true/yes/1 prefix (shd-topology.c:754-775) */
    top->prefer_direct = pref_val && (!strncasecmp(pref_val, "true", 4) || !strncasecmp(pref_val, "yes", 3) ||
                                      !strncasecmp(pref_val, "1", 1));
    if (pref_text) xmlFree(pref_text);

    const int32_t n = (int32_t)nm.n;
    top->n = n;
    top->m = (int64_t)ne;
    top->esrc = malloc((ne ? ne : 1) * sizeof(int32_t));
    top->edst = malloc((ne ? ne : 1) * sizeof(int32_t));
    top->elat = malloc((ne ? ne : 1) * sizeof(double));
    top->eloss = malloc((ne ? ne : 1) * sizeof(double));
    /* vertex attributes: keys by exact attr.name (igraph attribute names) */
    int vs_key[VS_COUNT], vn_key[VN_COUNT];
    for (int a = 0; a < VS_COUNT; ++a) vs_key[a] = -1;
    for (int a = 0; a < VN_COUNT; ++a) vn_key[a] = -1;
    for (size_t i = 0; i < nkeys; ++i) {
        if (!keys[i].name || !(keys[i].for_ == 1 || keys[i].for_ == 3)) continue;
        for (int a = 1; a < VS_COUNT; ++a)
            if (!strcmp(keys[i].name, VS_NAMES[a])) vs_key[a] = (int)i;
        for (int a = 0; a < VN_COUNT; ++a)
            if (!strcmp(keys[i].name, VN_NAMES[a])) vn_key[a] = (int)i;
    }
    top->vstr[VS_ID] = calloc((size_t)n + 1, sizeof(char*));
    for (int32_t v = 0; v < n; ++v) top->vstr[VS_ID][v] = strdup(nm.names[v]);
    for (int a = 1; a < VS_COUNT; ++a)
        if (vs_key[a] >= 0) {
            top->vstr[a] = calloc((size_t)n + 1, sizeof(char*));
            for (int32_t v = 0; v < n; ++v)
                top->vstr[a][v] = strdup(keys[vs_key[a]].def ? keys[vs_key[a]].def : "");
        }
    for (int a = 0; a < VN_COUNT; ++a)
        if (vn_key[a] >= 0) {
            top->vnum[a] = malloc(((size_t)n + 1) * sizeof(double));
            const double d = parse_num(keys[vn_key[a]].def);
            for (int32_t v = 0; v < n; ++v) top->vnum[a][v] = d;
        }
    for (size_t i = 0; i < nn; ++i) {
        const int32_t v = nodes[i].v;
        for (xmlNode* d = nodes[i].el->children; d; d = d->next) {
            if (d->type != XML_ELEMENT_NODE || xmlStrcmp(d->name, (const xmlChar*)"data")) continue;
            xmlChar* k = xmlGetProp(d, (const xmlChar*)"key");
            xmlChar* txt = xmlNodeGetContent(d);
            for (int a = 1; a < VS_COUNT; ++a)
                if (vs_key[a] >= 0 && k && !strcmp((const char*)k, keys[vs_key[a]].id)) {
                    free(top->vstr[a][v]);
                    top->vstr[a][v] = strdup(txt ? (const char*)txt : "");
                }
            for (int a = 0; a < VN_COUNT; ++a)
                if (vn_key[a] >= 0 && k && !strcmp((const char*)k, keys[vn_key[a]].id))
                    top->vnum[a][v] = parse_num((const char*)txt);
            xmlFree(k);
            xmlFree(txt);
        }
    }
    /* edges: latency / packetloss / jitter by exact name */
    int ek_lat = -1, ek_loss = -1, ek_jit = -1;
    for (size_t i = 0; i < nkeys; ++i) {
        if (!keys[i].name || !(keys[i].for_ == 2 || keys[i].for_ == 3)) continue;
        if (!strcmp(keys[i].name, "latency")) ek_lat = (int)i;
        if (!strcmp(keys[i].name, "packetloss")) ek_loss = (int)i;
        if (!strcmp(keys[i].name, "jitter")) ek_jit = (int)i;
    }
    /* attribute names and types (shd-topology.c:550-707; the per-vertex and
     * per-edge value checks below still need bandwidth / latency / loss values) */
    if (!check_attribute_types(top, keys, nkeys)) {
        tlog(top, LOG_CRITICAL, "topology validation failed because of problem with graph, vertex, or edge attributes");
        ok = 0;
    }
    size_t e = 0;
    for (xmlNode* c = graph->children; c; c = c->next) {
        if (c->type != XML_ELEMENT_NODE || xmlStrcmp(c->name, (const xmlChar*)"edge")) continue;
        xmlChar* s = xmlGetProp(c, (const xmlChar*)"source");
        xmlChar* t = xmlGetProp(c, (const xmlChar*)"target");
        top->esrc[e] = name_index(&nm, s ? (const char*)s : "");
        top->edst[e] = name_index(&nm, t ? (const char*)t : "");
        xmlFree(s);
        xmlFree(t);
        double lat = ek_lat >= 0 ? parse_num(keys[ek_lat].def) : NAN;
        double loss = ek_loss >= 0 ? parse_num(keys[ek_loss].def) : NAN;
        double jit = ek_jit >= 0 ? parse_num(keys[ek_jit].def) : NAN;
        for (xmlNode* d = c->children; d; d = d->next) {
            if (d->type != XML_ELEMENT_NODE || xmlStrcmp(d->name, (const xmlChar*)"data")) continue;
            xmlChar* k = xmlGetProp(d, (const xmlChar*)"key");
            xmlChar* txt = xmlNodeGetContent(d);
            if (k && ek_lat >= 0 && !strcmp((const char*)k, keys[ek_lat].id)) lat = parse_num((const char*)txt);
            if (k && ek_loss >= 0 && !strcmp((const char*)k, keys[ek_loss].id)) loss = parse_num((const char*)txt);
            if (k && ek_jit >= 0 && !strcmp((const char*)k, keys[ek_jit].id)) jit = parse_num((const char*)txt);
            xmlFree(k);
            xmlFree(txt);
        }
        /* _topology_checkGraphEdgesHelperHook, shd-topology.c:1026-1109 */
        if (!(lat > 0.0)) {
            tlog(top, LOG_WARNING, "required attribute 'latency' on edge %zu is non-positive, missing or NAN", e);
            ok = 0;
        }
        if (!(loss >= 0.0 && loss <= 1.0)) {
            tlog(top, LOG_WARNING, "required attribute 'packetloss' on edge %zu is out of range or missing", e);
            ok = 0;
        }
        if (!isnan(jit) && !(jit >= 0.0)) {
            tlog(top, LOG_WARNING, "optional attribute 'jitter' on edge %zu is negative", e);
            ok = 0;
        }
        top->elat[e] = lat;
        top->eloss[e] = loss;
        e++;
    }
    /* _topology_checkGraphVerticesHelperHook, shd-topology.c:796-963 */
    for (int32_t v = 0; v < n && ok; ++v) {
        if (!top->vnum[VN_BWDOWN] || !top->vnum[VN_BWUP]) {   /* :828-862 "is missing" */
            tlog(top, LOG_WARNING, "required bandwidth attribute on vertex %d ('%s') is missing", v,
                 top->vstr[VS_ID][v]);
            ok = 0;
        } else if (!(top->vnum[VN_BWDOWN][v] > 0.0) || !(top->vnum[VN_BWUP][v] > 0.0)) {
            tlog(top, LOG_WARNING, "required bandwidth attribute on vertex %d ('%s') is NAN or negative", v,
                 top->vstr[VS_ID][v]);
            ok = 0;
        }
        if (top->vnum[VN_ASN] && !isnan(top->vnum[VN_ASN][v]) && !(top->vnum[VN_ASN][v] > 0.0)) {
            tlog(top, LOG_WARNING, "optional attribute 'asn' on vertex %d is non-positive", v);
            ok = 0;
        }
        const double pl = top->vnum[VN_PACKETLOSS] ? top->vnum[VN_PACKETLOSS][v] : NAN;
        if (!isnan(pl) && !(pl >= 0.0 && pl <= 1.0)) {
            tlog(top, LOG_WARNING, "optional attribute 'packetloss' on vertex %d is out of range [0.0,1.0]", v);
            ok = 0;
        }
    }
    free(nodes);
    for (size_t i = 0; i < nm.n; ++i) free(nm.names[i]);
    free(nm.names);
    free(nm.hkeys);
    free(nm.hvals);
out:
    for (size_t i = 0; i < nkeys; ++i) {
        free(keys[i].id);
        free(keys[i].name);
        free(keys[i].def);
    }
    free(keys);
    xmlFreeDoc(doc);
    return ok;
}

/* one strong component (igraph_is_connected STRONG + clusters == 1, :723-791) */
static int strongly_connected(const Topology* top) {
    const int32_t n = top->n;
    if (n <= 1) return 1;
    int32_t* deg = calloc((size_t)n + 1, sizeof(int32_t));
    int32_t* rdeg = calloc((size_t)n + 1, sizeof(int32_t));
    for (int64_t e = 0; e < top->m; ++e) {
        deg[top->esrc[e] + 1]++;
        rdeg[top->edst[e] + 1]++;
        if (!top->directed) {
            deg[top->edst[e] + 1]++;
            rdeg[top->esrc[e] + 1]++;
        }
    }
    for (int32_t v = 0; v < n; ++v) {
        deg[v + 1] += deg[v];
        rdeg[v + 1] += rdeg[v];
    }
    int32_t* adj = malloc(((size_t)deg[n] + 1) * sizeof(int32_t));
    int32_t* radj = malloc(((size_t)rdeg[n] + 1) * sizeof(int32_t));
    int32_t* fill = calloc((size_t)n, sizeof(int32_t));
    int32_t* rfill = calloc((size_t)n, sizeof(int32_t));
    for (int64_t e = 0; e < top->m; ++e) {
        const int32_t a = top->esrc[e], b = top->edst[e];
        adj[deg[a] + fill[a]++] = b;
        radj[rdeg[b] + rfill[b]++] = a;
        if (!top->directed) {
            adj[deg[b] + fill[b]++] = a;
            radj[rdeg[a] + rfill[a]++] = b;
        }
    }
    int32_t* stack = malloc((size_t)n * sizeof(int32_t));
    uint8_t* seen = calloc((size_t)n, 1);
    int ok = 1;
    for (int pass = 0; pass < 2 && ok; ++pass) {
        const int32_t* P = pass ? rdeg : deg;
        const int32_t* E = pass ? radj : adj;
        memset(seen, 0, (size_t)n);
        int32_t sp = 0, cnt = 1;
        stack[sp++] = 0;
        seen[0] = 1;
        while (sp) {
            const int32_t x = stack[--sp];
            for (int32_t k = P[x]; k < P[x + 1]; ++k)
                if (!seen[E[k]]) {
                    seen[E[k]] = 1;
                    cnt++;
                    stack[sp++] = E[k];
                }
        }
        ok = cnt == n;
    }
    free(deg); free(rdeg); free(adj); free(radj); free(fill); free(rfill); free(stack); free(seen);
    return ok;
}

/* --------------------------------------------------------- lifecycle */

static uint32_t string_to_ip(const char* s) {   /* address_stringToIP, shd-address.c:137-144 */
    struct in_addr a;
    if (s && inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return INADDR_NONE;
}

static int cmp_u64(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* the whole-table host mirror (tens of GB): anonymous pages, transparent huge pages
 * asked for, so filling it faults 2-MB pages instead of 4-KB ones */
static void* big_alloc(size_t bytes) {
    void* p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return NULL;
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    return p;
}

static void big_free(void* p, size_t bytes) {
    if (p) munmap(p, bytes);
}

/* Page faults of a fresh tens-of-GB mirror cost seconds on a host without free huge
 * pages; touching its pages on several threads while the GPU builds the table hides
 * them behind the build (pre_touch_start before spe_table_build, _join after). */
typedef struct {
    char* p;
    size_t a, b;
} TouchJob;

static void* touch_pages(void* x) {
    TouchJob* j = x;
    for (size_t i = j->a; i < j->b; i += 4096) ((volatile char*)j->p)[i] = 0;
    return NULL;
}

enum { TOUCH_MAX = 32 };
typedef struct {
    pthread_t th[TOUCH_MAX];
    TouchJob job[TOUCH_MAX];
    int started[TOUCH_MAX];
    int n;
} PreTouch;

static int host_cpus(void);

static void pre_touch_start(PreTouch* pt, char* p0, char* p1, size_t bytes) {
    memset(pt, 0, sizeof *pt);
    int n = host_cpus();
    if (n > TOUCH_MAX) n = TOUCH_MAX;
    if (n < 2) n = 2;
    pt->n = n;
    for (int k = 0; k < n; ++k) {   /* half the threads per array */
        char* p = k % 2 ? p1 : p0;
        const int h = k / 2, H = (n + 1 - k % 2) / 2;
        pt->job[k] = (TouchJob){p, bytes * (size_t)h / (size_t)H & ~(size_t)4095, bytes * (size_t)(h + 1) / (size_t)H};
        pt->started[k] = pthread_create(&pt->th[k], NULL, touch_pages, &pt->job[k]) == 0;
    }
}

static void pre_touch_join(PreTouch* pt) {
    for (int k = 0; k < pt->n; ++k) {
        if (pt->started[k]) pthread_join(pt->th[k], NULL);
        else touch_pages(&pt->job[k]);
    }
}

static void snap_free(Snap* s) {
    if (!s) return;
    if (s->table) spe_table_free(s->table);
    if (s->blocks) {
        for (int32_t b = 0; b < s->A; ++b) free(atomic_load(&s->blocks[b]));
        free(s->blocks);
        free((void*)s->touch);
    }
    big_free(s->mlat, (size_t)s->A * s->A * sizeof(double));
    big_free(s->mrel, (size_t)s->A * s->A * sizeof(double));
    free(s->slot_of_vertex);
    free(s->attached);
    pthread_mutex_destroy(&s->row_mu);
    free(s);
}

static void topo_release(Topology* top) {
    if (!top) return;
    snap_free(top->snap);
    if (top->graph) spe_graph_free(top->graph);
    for (int a = 0; a < VS_COUNT; ++a)
        if (top->vstr[a]) {
            for (int32_t v = 0; v < top->n; ++v) free(top->vstr[a][v]);
            free(top->vstr[a]);
        }
    for (int a = 0; a < VN_COUNT; ++a) free(top->vnum[a]);
    free(top->esrc); free(top->edst); free(top->elat); free(top->eloss);
    free(top->vip); free(top->vip_index);
    free(top->ips);
    free(top->is_attached); free(top->attached);
    free((void*)top->run_seq);
    free((void*)top->xflag);
    for (int i = 0; i < NSHARD; ++i) {
        free(top->shards[i].tab);
        pthread_mutex_destroy(&top->shards[i].mu);
    }
    state_destroy(top);
    pthread_mutex_destroy(&top->seal_lock);
    pthread_mutex_destroy(&top->cache_mu);
    pthread_mutex_destroy(&top->batch_mu);
    free(top->bscr);
    free(top);
}

Topology* topology_new_on_device(const char* graphPath, int32_t device) {
    if (!graphPath) return NULL;
    Topology* top = calloc(1, sizeof(Topology));
    top->device = device;
    top->log_level = LOG_MESSAGE;
    state_init(top);
    pthread_mutex_init(&top->seal_lock, NULL);
    pthread_mutex_init(&top->cache_mu, NULL);
    pthread_mutex_init(&top->batch_mu, NULL);
    for (int i = 0; i < NSHARD; ++i) pthread_mutex_init(&top->shards[i].mu, NULL);
    const char* mode = getenv("SHADOW_SPE_PATH_CACHE");
    top->cache_mode = (mode && !strcasecmp(mode, "reference")) ? TOPOLOGY_ANSWER_REFERENCE : TOPOLOGY_ANSWER_ROWS;
    tlog(top, LOG_MESSAGE, "reading graphml topology graph at '%s'...", graphPath);
    if (!load_graphml(top, graphPath) || !strongly_connected(top)) {
        tlog(top, LOG_CRITICAL, "we failed to create the simulation topology because we were unable to "
                                "validate the topology graphml file");
        topo_release(top);
        return NULL;
    }
    double* vloss = top->vnum[VN_PACKETLOSS];
    double* nanv = NULL;
    if (!vloss) {
        nanv = malloc(((size_t)top->n + 1) * sizeof(double));
        for (int32_t v = 0; v < top->n; ++v) nanv[v] = NAN;
    }
    spe_graph_desc d = {sizeof(spe_graph_desc), top->n, top->m, top->esrc, top->edst, top->elat, top->eloss, vloss ? vloss : nanv,
                        top->directed, top->prefer_direct};
    const int rc = spe_graph_create(&d, device, &top->graph);
    free(nanv);
    if (rc != SPE_OK) {
        tlog(top, LOG_CRITICAL, "spe_graph_create failed: %s", spe_last_error());
        topo_release(top);
        return NULL;
    }
    spe_graph_info info = SPE_STRUCT_INIT(spe_graph_info);
    spe_graph_info_get(top->graph, &info);
    top->complete = info.complete;
    top->shared_rows_exact = info.shared_rows_exact;
    if (!info.weight_floor_ok)   /* outside the bit-exactness argument */
        tlog(top, LOG_WARNING, "some edge latency is below ulp(path latency)/2: a relaxation could leave a "
                               "distance unchanged (fl(d + w) == d); routes are exact only when every "
                               "fl(d + w) > d");
    tlog(top, LOG_MESSAGE, "topology graph is %s, %s, and strongly connected with 1 cluster. It does%s prefer "
                           "direct paths.", info.complete ? "complete" : "incomplete",
         top->directed ? "directed" : "undirected", top->prefer_direct ? "" : " not");
    /* every vertex's ip parsed once; the usable ones indexed by (ip, vertex) */
    top->vip = malloc(((size_t)top->n + 1) * sizeof(uint32_t));
    top->vip_index = malloc(((size_t)top->n + 1) * sizeof(uint64_t));
    for (int32_t v = 0; v < top->n; ++v) {
        const uint32_t ip = string_to_ip(top->vstr[VS_IP] ? top->vstr[VS_IP][v] : NULL);
        top->vip[v] = ip;
        if (ip != INADDR_NONE && ip != INADDR_ANY && ip != INADDR_LOOPBACK)
            top->vip_index[top->n_vip++] = ((uint64_t)ip << 32) | (uint32_t)v;
    }
    qsort(top->vip_index, (size_t)top->n_vip, sizeof(uint64_t), cmp_u64);
    top->ip_cap = 1024;
    top->ips = malloc(top->ip_cap * sizeof(IpSlot));
    for (size_t i = 0; i < top->ip_cap; ++i) top->ips[i] = (IpSlot){0, IP_EMPTY};
    top->is_attached = calloc((size_t)top->n + 1, 1);
    top->attached = malloc(((size_t)top->n + 1) * sizeof(int32_t));
    top->run_seq = calloc((size_t)top->n + 1, sizeof(uint64_t));
    top->xflag = calloc((size_t)top->n + 1, sizeof(uint8_t));
    return top;
}

int32_t topology_check_graphml(const char* graphPath) {
    if (!graphPath) return 0;
    Topology* top = calloc(1, sizeof(Topology));
    top->log_level = LOG_WARNING;
    state_init(top);
    pthread_mutex_init(&top->seal_lock, NULL);
    pthread_mutex_init(&top->cache_mu, NULL);
    pthread_mutex_init(&top->batch_mu, NULL);
    for (int i = 0; i < NSHARD; ++i) pthread_mutex_init(&top->shards[i].mu, NULL);
    const int ok = load_graphml(top, graphPath) && strongly_connected(top);
    topo_release(top);
    return ok ? 1 : 0;
}

Topology* topology_new(const char* graphPath) {
    /* SHADOW_SPE_DEVICE=<index>: the GPU to build on (default 0) */
    const char* dev = getenv("SHADOW_SPE_DEVICE");
    return topology_new_on_device(graphPath, dev && *dev ? atoi(dev) : 0);
}

void topology_set_log_callback(Topology* top, topology_log_fn fn, void* ctx) {
    if (!top) return;
    top->log_fn = fn;
    top->log_ctx = ctx;
}

void topology_set_log_level(Topology* top, int32_t level) {
    if (top) top->log_level = level;
}

void topology_set_min_latency_callback(Topology* top, topology_min_latency_fn fn, void* ctx) {
    if (!top) return;
    top->minlat_fn = fn;
    top->minlat_ctx = ctx;
}

int32_t topology_set_answer_mode(Topology* top, int32_t mode) {
    if (!top || (mode != TOPOLOGY_ANSWER_ROWS && mode != TOPOLOGY_ANSWER_REFERENCE)) return SPE_EINVAL;
    top->cache_mode = mode;
    return SPE_OK;
}

int32_t topology_vertex_count(const Topology* top) { return top ? top->n : 0; }

/* ----------------------------------------------------- IP -> vertex map */

/* 64-bit finaliser (every input bit reaches the low bits the tables index by):
 * in_addr_t values are in network byte order, so on a little-endian host a
 * plain multiplicative hash's low bits saw only the first octets -- every host of
 * a 10.x.y.z plan in one probe chain */
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

static uint64_t hash_ip(uint32_t ip) { return mix64(ip); }

static void ip_put(Topology* top, uint32_t ip, int32_t v) {
    if ((top->ip_size + 1) * 2 > top->ip_cap) {   /* grow (detached slots are dropped) */
        const size_t nc = top->ip_cap * 2;
        IpSlot* n = malloc(nc * sizeof(IpSlot));
        for (size_t i = 0; i < nc; ++i) n[i] = (IpSlot){0, IP_EMPTY};
        size_t live = 0;
        for (size_t i = 0; i < top->ip_cap; ++i)
            if (top->ips[i].v >= 0) {
                size_t j = hash_ip(top->ips[i].ip) & (nc - 1);
                while (n[j].v != IP_EMPTY) j = (j + 1) & (nc - 1);
                n[j] = top->ips[i];
                ++live;
            }
        free(top->ips);
        top->ips = n;
        top->ip_cap = nc;
        top->ip_size = live;
    }
    size_t j = hash_ip(ip) & (top->ip_cap - 1);
    while (top->ips[j].v != IP_EMPTY) {
        if (top->ips[j].v >= 0 && top->ips[j].ip == ip) {
            top->ips[j].v = v;
            return;
        }
        j = (j + 1) & (top->ip_cap - 1);
    }
    top->ips[j] = (IpSlot){ip, v};
    top->ip_size++;
}

static int32_t ip_get(const Topology* top, uint32_t ip) {
    size_t j = hash_ip(ip) & (top->ip_cap - 1);
    for (IpSlot x; (x = top->ips[j]).v != IP_EMPTY; j = (j + 1) & (top->ip_cap - 1))
        if (x.v >= 0 && x.ip == ip) return x.v;
    return -1;
}

static void ip_del(Topology* top, uint32_t ip) {
    size_t j = hash_ip(ip) & (top->ip_cap - 1);
    while (top->ips[j].v != IP_EMPTY) {
        if (top->ips[j].v >= 0 && top->ips[j].ip == ip) {
            top->ips[j].v = IP_GONE;   /* tombstone: probes continue past it */
            return;
        }
        j = (j + 1) & (top->ip_cap - 1);
    }
}

/* ---------------------------------------------------------- attachment */

typedef struct {
    int32_t* q;
    size_t n;
    uint32_t nips;
} Cand;

static void cand_push(Cand* c, int32_t v, int usable, size_t cap) {
    if (!c->q) c->q = malloc(cap * sizeof(int32_t));
    c->q[c->n++] = v;
    if (usable) c->nips++;
}

static int str_match(const char* attr, const char* hint) {   /* found && hint && !g_ascii_strcasecmp */
    return attr && attr[0] != '\0' && hint && !strcasecmp(attr, hint);
}

/* _topology_findAttachmentVertex + hook, shd-topology.c:2077-2352 */
static int32_t find_attachment_vertex(Topology* top, topology_random_fn rnd, void* rctx, const char* ipHint,
                                      const char* cityHint, const char* countryHint, const char* geoHint,
                                      const char* typeHint) {
    enum { C_CITYTYPE = 0, C_CITY, C_COUNTRYTYPE, C_COUNTRY, C_GEOTYPE, C_GEO, C_TYPE, C_ALL, C_N };
    Cand c[C_N];
    memset(c, 0, sizeof c);
    const size_t cap = (size_t)top->n + 1;
    int requestedUsable = 0, foundExact = 0;
    uint32_t requestedIP = 0;
    if (ipHint) {
        const uint32_t ip = string_to_ip(ipHint);
        if (ip != INADDR_NONE && ip != INADDR_ANY && ip != INADDR_LOOPBACK) {
            requestedUsable = 1;
            requestedIP = ip;
        }
    }
    if (requestedUsable && top->vip_index) {
        /* Vertices whose ip equals the hint: the scan below would clear every queue at
         * the first of them and keep exactly these, in vertex order, then pick one at
         * random (no longest-prefix match once an exact one was found).  The sorted
         * index finds them without the O(n) scan (a 100k-host attach on a 200k-vertex
         * graph would otherwise be 2e10 string compares). */
        int64_t lo = 0, hi = top->n_vip;
        const uint64_t key = (uint64_t)requestedIP << 32;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (top->vip_index[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        int64_t e = lo;
        while (e < top->n_vip && (uint32_t)(top->vip_index[e] >> 32) == requestedIP) ++e;
        if (e > lo) {
            const double r = rnd ? rnd(rctx) : 0.0;
            const int indexRange = (int)(e - lo) - 1;
            int idx = (int)round((double)(indexRange * r));   /* :2310-2316 */
            if (idx < 0) idx = 0;
            if (idx > indexRange) idx = indexRange;
            return (int32_t)(uint32_t)top->vip_index[lo + idx];
        }
    }
    for (int32_t v = 0; v < top->n; ++v) {
        const char* city = top->vstr[VS_CITYCODE] ? top->vstr[VS_CITYCODE][v] : NULL;
        const char* country = top->vstr[VS_COUNTRYCODE] ? top->vstr[VS_COUNTRYCODE][v] : NULL;
        const char* geo = top->vstr[VS_GEOCODE] ? top->vstr[VS_GEOCODE][v] : NULL;
        const char* type = top->vstr[VS_TYPE] ? top->vstr[VS_TYPE][v] : NULL;
        const int cityM = str_match(city, cityHint), countryM = str_match(country, countryHint);
        const int geoM = str_match(geo, geoHint), typeM = str_match(type, typeHint);
        const uint32_t vip = top->vip[v];
        const int usable = vip != INADDR_NONE && vip != INADDR_ANY && vip != INADDR_LOOPBACK;
        if (requestedUsable && usable && vip == requestedIP) {
            if (!foundExact)   /* g_queue_clear on every queue; the numIPs counters are kept */
                for (int i = 0; i < C_N; ++i) c[i].n = 0;
            foundExact = 1;
            cand_push(&c[C_ALL], v, usable, cap);
        }
        if (foundExact) continue;
        cand_push(&c[C_ALL], v, usable, cap);
        if (cityM && typeM) cand_push(&c[C_CITYTYPE], v, usable, cap);
        if (cityM) cand_push(&c[C_CITY], v, usable, cap);
        if (countryM && typeM) cand_push(&c[C_COUNTRYTYPE], v, usable, cap);
        if (countryM) cand_push(&c[C_COUNTRY], v, usable, cap);
        if (geoM && typeM) cand_push(&c[C_GEOTYPE], v, usable, cap);
        if (geoM) cand_push(&c[C_GEO], v, usable, cap);
        if (typeM) cand_push(&c[C_TYPE], v, usable, cap);
    }
    Cand* pick = NULL;
    int lpm = 0;
    for (int i = 0; i < C_ALL && !pick; ++i)
        if (c[i].n > 0) {
            pick = &c[i];
            lpm = requestedUsable && c[i].nips > 0;
        }
    if (!pick) {
        pick = &c[C_ALL];
        lpm = ipHint && c[C_ALL].nips > 0;
    }
    int32_t chosen = -1;
    if (pick->n > 0) {
        if (lpm && !foundExact) {   /* _topology_getLongestPrefixMatch, :2202-2229 */
            uint32_t best = 0;
            for (size_t i = 0; i < pick->n; ++i) {
                const int32_t v = pick->q[i];
                const uint32_t vip = top->vip[v];
                const uint32_t match = vip & requestedIP;
                if (match > best) {
                    best = match;
                    chosen = v;
                }
            }
        } else {
            const double r = rnd ? rnd(rctx) : 0.0;
            const int indexRange = (int)pick->n - 1;
            const int idx = (int)round((double)(indexRange * r));   /* :2310-2316 */
            chosen = pick->q[idx < 0 ? 0 : (idx >= (int)pick->n ? (int)pick->n - 1 : idx)];
        }
    }
    for (int i = 0; i < C_N; ++i) free(c[i].q);
    return chosen;
}

void topology_attach(Topology* top, spe_in_addr_t address, topology_random_fn random, void* random_ctx,
                     const char* ipHint, const char* citycodeHint, const char* countrycodeHint,
                     const char* geocodeHint, const char* typeHint, uint64_t* bwDownOut, uint64_t* bwUpOut) {
    if (!top) return;
    const int32_t v = find_attachment_vertex(top, random, random_ctx, ipHint, citycodeHint, countrycodeHint,
                                             geocodeHint, typeHint);
    if (v < 0) {
        tlog(top, LOG_CRITICAL, "unable to find an attachment vertex");
        return;
    }
    /* A new vertex only joins the attached set here; a sealed table stays
     * published (it answers every pair it holds) until the next query that needs
     * the new vertex builds and publishes a replacement. */
    state_wrlock(top);
    ip_put(top, address, v);
    if (!top->is_attached[v]) {
        top->is_attached[v] = 1;
        top->attached[top->n_attached++] = v;
    }
    state_wrunlock(top);
    if (bwUpOut) *bwUpOut = (uint64_t)top->vnum[VN_BWUP][v];
    if (bwDownOut) *bwDownOut = (uint64_t)top->vnum[VN_BWDOWN][v];
    struct in_addr a = {address};
    tlog(top, LOG_MESSAGE, "attached address '%s' to vertex %d ('%s')", inet_ntoa(a), v, top->vstr[VS_ID][v]);
}

void topology_detach(Topology* top, spe_in_addr_t address) {
    if (!top) return;
    state_wrlock(top);
    ip_del(top, address);   /* the vertex stays in A, like the reference (:2415-2421) */
    state_wrunlock(top);
}

int32_t topology_attached_vertex(const Topology* top, spe_in_addr_t address) {
    if (!top) return -1;
    state_rdlock(top);
    const int32_t v = ip_get((Topology*)top, address);
    state_rdunlock(top);
    return v;
}

/* -------------------------------------------------------------- sealing */

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int64_t env_bytes(const char* name, int64_t dflt) {
    const char* s = getenv(name);
    return (s && *s) ? (int64_t)strtoll(s, NULL, 10) : dflt;
}

/* Host-mirror budget: SHADOW_SPE_MIRROR_BYTES, else min(48 GiB, half of the host's
 * available memory) -- the whole record span of a 50k-host table (40 GB) where the
 * host has the room.  A re-seal fills the new mirror while the published one is
 * still held: MemAvailable already excludes what it holds, a fixed cap does not,
 * so `held` is subtracted from a fixed cap only (*fixed = 1) and handed back to
 * the new snapshot once the old one is freed (topology_seal). */
static int64_t mem_available_bytes(void) {
    FILE* f = fopen("/proc/meminfo", "r");
    if (!f) return -1;
    char line[256];
    int64_t kb = -1;
    while (fgets(line, sizeof line, f))
        if (sscanf(line, "MemAvailable: %lld kB", (long long*)&kb) == 1) break;
    fclose(f);
    return kb < 0 ? -1 : kb * 1024;
}

static int64_t mirror_budget(int64_t held, int* fixed) {
    const char* e = getenv("SHADOW_SPE_MIRROR_BYTES");
    const int64_t avail = mem_available_bytes();
    *fixed = (e && *e) || avail <= 0;
    if (*fixed) return env_bytes("SHADOW_SPE_MIRROR_BYTES", (int64_t)8 << 30) - held;
    const int64_t cap = (int64_t)48 << 30;
    return avail / 2 < cap ? avail / 2 : cap;
}

/* bytes of host mirror a snapshot holds */
static int64_t snap_mirror_bytes(const Snap* s) {
    if (!s) return 0;
    if (s->mlat) return (int64_t)s->A * s->A * 16;
    return s->blocks ? s->mirror_budget - atomic_load(&s->row_budget) : 0;
}

static int snap_build(Topology* top, const int32_t* att_in, int32_t A, int64_t budget, Snap** out) {
    *out = NULL;
    /* SHADOW_SPE_SEAL_TIMING: one stderr line of the seal's phases */
    const int timing = getenv("SHADOW_SPE_SEAL_TIMING") != NULL;
    double tp[8] = {0};
    int np = 0;
    if (timing) tp[np++] = now_s();
    Snap* s = calloc(1, sizeof(Snap));
    pthread_mutex_init(&s->row_mu, NULL);
    atomic_store(&s->host_reads, -1);
    s->A = A;
    s->attached = malloc(((size_t)A + 1) * sizeof(int32_t));
    s->slot_of_vertex = malloc(((size_t)top->n + 1) * sizeof(int32_t));
    for (int32_t v = 0; v < top->n; ++v) s->slot_of_vertex[v] = -1;
    /* slots are internal (queries resolve IP -> vertex -> slot): number them in
     * the engine's source-clustering order (spe_order_sources) */
    if (spe_order_sources(top->graph, att_in, A, s->attached) != SPE_OK)
        memcpy(s->attached, att_in, (size_t)A * sizeof(int32_t));
    for (int32_t i = 0; i < A; ++i) s->slot_of_vertex[s->attached[i]] = i;
    spe_table_opts o;
    memset(&o, 0, sizeof o);
    o.struct_size = sizeof o;
    o.self_mode = SPE_SELF_ROW;
    /* SHADOW_SPE_DEVICES=0,1,...: build on several GPUs of this node (one share of
     * the sources each, then an all-gather of the records, spe_table_opts.devices) */
    int32_t devs[64];
    int32_t ndev = 0;
    const char* dl = getenv("SHADOW_SPE_DEVICES");
    for (const char* p = dl; p && *p && ndev < 64;) {
        char* end = NULL;
        const long d = strtol(p, &end, 10);
        if (end == p) break;
        devs[ndev++] = (int32_t)d;
        p = (*end == ',') ? end + 1 : end;
    }
    if (ndev > 1) {
        o.devices = devs;
        o.n_devices = ndev;
    }
    /* SHADOW_SPE_ENGINE=1|2|3: ask for the batch / LDS / FW engine (SPE_ENGINE_*); an
     * engine the graph does not fit falls back to the library's choice */
    const char* eng = getenv("SHADOW_SPE_ENGINE");
    if (eng && *eng) o.engine = (int32_t)strtol(eng, NULL, 10);
    /* Every host on its own relaxation lane unless every path sum is exact in f64.
     * Shadow turns a latency into simulated time as ceil(latency * 1e6) ns
     * (shd-worker.c:244), and real topologies carry decimal latencies (the shipped
     * one: 5.0 .. 2293.85 ms), whose products sit on or next to an integer: the few
     * ulps by which a shared / derived row differs from the path-order sum
     *  would move a delivery by 1 ns.  So the drop-in's default is
     * bit-exact: shared anchor trees and derived rows only where every path sum AND
     * every reliability product is exact (spe_graph_info.shared_rows_exact: latencies
     * k / 2^q, e.g. integers, and no edge loss -- a shared row multiplies
     * a(s, c) * r_c(t) where the reference folds from the source), where
     * they equal the exact build bit for bit.  SHADOW_SPE_EXACT_SOURCES=0 / 1
     * overrides it either way. */
    const char* ex = getenv("SHADOW_SPE_EXACT_SOURCES");
    o.exact_sources = top->shared_rows_exact ? 0 : 1;
    if (ex && *ex) o.exact_sources = strcmp(ex, "0") != 0;
    if (timing) tp[np++] = now_s();   /* slot order */
    int rc = spe_table_create(top->graph, s->attached, A, &o, &s->table);
    if (rc == SPE_EUNSUPPORTED && o.engine != SPE_ENGINE_AUTO) {
        o.engine = SPE_ENGINE_AUTO;
        rc = spe_table_create(top->graph, s->attached, A, &o, &s->table);
    }
    if (timing) tp[np++] = now_s();   /* table create: device memory */
    /* SHADOW_SPE_TABLE_CACHE=<dir>: reuse the rows of an earlier run on the same
     * graph / hosts (keyed file), else build and save them */
    const char* cdir = getenv("SHADOW_SPE_TABLE_CACHE");
    char cpath[4096] = {0};
    int loaded = 0;
    if (rc == SPE_OK && cdir && *cdir && ndev <= 1) {   /* the cache holds single-device tables */
        uint64_t key = 0;
        spe_table_key(s->table, &key);
        snprintf(cpath, sizeof cpath, "%s/spe-table-%016llx.bin", cdir, (unsigned long long)key);
        loaded = spe_table_load(s->table, cpath) == SPE_OK;
        tlog(top, LOG_MESSAGE, "path table cache %s: %s", loaded ? "hit" : "miss", cpath);
    }
    /* host view: the whole table when it fits the mirror budget (mirror_budget: up to
     * 48 GiB, A <= 56k; spe_table_download streams it through pinned staging), else
     * source rows mirrored once they are read repeatedly, within that budget, and
     * single-record device reads (spe_table_get_latrel) otherwise; batches of queries
     * read the device table in one launch (topology_getPathInfoBatch).  The whole-table
     * mirror is allocated first and its pages touched while the GPU builds. */
    if (budget < 0) budget = 0;
    s->mirror_budget = budget;
    const int64_t full = (int64_t)A * A * 16;
    PreTouch pt;
    int touching = 0;
    if (rc == SPE_OK && full <= budget) {
        s->mlat = big_alloc((size_t)A * A * sizeof(double));
        s->mrel = big_alloc((size_t)A * A * sizeof(double));
        if (!s->mlat || !s->mrel) rc = SPE_ENOMEM;
        else {
            pre_touch_start(&pt, (char*)s->mlat, (char*)s->mrel, (size_t)A * A * sizeof(double));
            touching = 1;
        }
    }
    if (timing) tp[np++] = now_s();   /* mirror allocation */
    if (rc == SPE_OK && !loaded) {
        rc = spe_table_build(s->table, NULL);
        if (rc == SPE_OK && cpath[0] && spe_table_save(s->table, cpath) != SPE_OK)
            tlog(top, LOG_WARNING, "could not save the path table cache: %s", spe_last_error());
    }
    if (timing) tp[np++] = now_s();   /* build */
    if (touching) pre_touch_join(&pt);
    if (timing) tp[np++] = now_s();   /* rest of the mirror's page touching */
    if (rc == SPE_OK && full <= budget) {
        rc = spe_table_download(s->table, 0, A, s->mlat, s->mrel, NULL, NULL);
    } else if (rc == SPE_OK) {
        s->blocks = calloc((size_t)A, sizeof(*s->blocks));
        s->touch = calloc((size_t)A, sizeof(*s->touch));
        atomic_store(&s->row_budget, budget);
        if (!s->blocks || !s->touch) rc = SPE_ENOMEM;
        double l0, r0;   /* the first read decides host reads and starts the library's pre-fault
                          * of the table's host mapping (spe_table_layout.host_prefault) now */
        if (rc == SPE_OK && spe_table_get_latrel(s->table, 0, 0, &l0, &r0) == SPE_OK) {
            spe_table_layout l;
            memset(&l, 0, sizeof l);
            l.struct_size = sizeof l;
            if (spe_table_layout_get(s->table, &l) == SPE_OK) atomic_store(&s->host_reads, l.host_reads);
        }
    }
    if (timing) tp[np++] = now_s();   /* download / first read */
    if (rc == SPE_OK) rc = spe_table_min_latency(s->table, &s->min_latency);
    if (timing) {
        tp[np++] = now_s();
        fprintf(stderr, "[topology] seal of %d hosts: order %.3f s, create %.3f s, mirror alloc %.3f s, build %.3f s, "
                        "touch wait %.3f s, download %.3f s, min latency %.3f s\n", A, tp[1] - tp[0], tp[2] - tp[1],
                tp[3] - tp[2], tp[4] - tp[3], tp[5] - tp[4], tp[6] - tp[5], tp[7] - tp[6]);
    }
    if (rc != SPE_OK) {
        tlog(top, LOG_CRITICAL, "path table build failed: %s", spe_last_error());
        snap_free(s);
        return rc;
    }
    *out = s;
    return SPE_OK;
}

int32_t topology_seal(Topology* top) {
    if (!top) return SPE_EINVAL;
    pthread_mutex_lock(&top->seal_lock);
    state_rdlock(top);
    const int32_t A = top->n_attached;
    const int fresh = top->snap && top->snap->A == A;   /* A only grows */
    int32_t* att = fresh ? NULL : malloc(((size_t)A + 1) * sizeof(int32_t));
    if (att) memcpy(att, top->attached, (size_t)A * sizeof(int32_t));
    state_rdunlock(top);
    int rc = SPE_OK;
    int64_t held = 0;
    int fixed = 0;
    if (!fresh) {
        Snap* s = NULL;
        if (A == 0) {
            rc = SPE_ESTATE;
        } else {
            const double t0 = now_s();
            /* the published snapshot's mirror stays allocated until the swap below */
            state_rdlock(top);
            held = snap_mirror_bytes(top->snap);
            state_rdunlock(top);
            rc = snap_build(top, att, A, mirror_budget(held, &fixed), &s);   /* no lock held: queries on the old table go on */
            if (rc == SPE_OK) {
                top->build_seconds += now_s() - t0;
                top->build_rows += A;
            }
        }
        if (rc == SPE_OK) {
            state_wrlock(top);   /* drains every reader of the old table */
            Snap* old = top->snap;
            top->snap = s;
            state_wrunlock(top);
            snap_free(old);
            if (fixed && held > 0 && s->blocks) {   /* the old mirror's bytes are free again */
                atomic_fetch_add(&s->row_budget, held);
                s->mirror_budget += held;
            }
            /* worker_updateMinTimeJump(minimumPathLatency), shd-topology.c:1359-1370: on the
             * querying (worker) thread, as the reference requires */
            if (top->cache_mode == TOPOLOGY_ANSWER_ROWS && top->minlat_fn && s->min_latency > 0)
                top->minlat_fn(s->min_latency, top->minlat_ctx);
        }
    }
    free(att);
    pthread_mutex_unlock(&top->seal_lock);
    return rc;
}

/* Latency and reliability of table entry (s, t) of a published snapshot; the
 * caller holds the state lock shared.  A source row is mirrored on its
 * ROW_MIRROR_AFTER-th single read, or its ROW_MIRROR_AFTER_HOST-th when the table
 * answers single entries with host loads (spe_table_layout.host_reads: ~2.6 us per
 * record, where a row's copy costs ~50 of them at A = 100k). */
#define ROW_MIRROR_AFTER 4
#define ROW_MIRROR_AFTER_HOST 64

static void snap_value(Topology* top, Snap* sn, int32_t s, int32_t t, double* lat, double* rel) {
    const int32_t A = sn->A;
    if (sn->mlat) {
        *lat = sn->mlat[(size_t)s * A + t];
        *rel = sn->mrel[(size_t)s * A + t];
        return;
    }
    const int64_t bytes = (int64_t)A * 16;
    double* row = atomic_load_explicit(&sn->blocks[s], memory_order_acquire);
    const int after = atomic_load_explicit(&sn->host_reads, memory_order_relaxed) == 1 ? ROW_MIRROR_AFTER_HOST
                                                                                       : ROW_MIRROR_AFTER;
    if (!row && atomic_load_explicit(&sn->touch[s], memory_order_relaxed) < 255 &&
        atomic_fetch_add(&sn->touch[s], 1) + 1 >= after && atomic_load(&sn->row_budget) >= bytes) {
        pthread_mutex_lock(&sn->row_mu);
        row = atomic_load_explicit(&sn->blocks[s], memory_order_acquire);
        if (!row && atomic_load(&sn->row_budget) >= bytes) {
            row = malloc((size_t)bytes);
            if (row && spe_table_get_row_latrel(sn->table, s, row, row + A) == SPE_OK) {
                atomic_fetch_sub(&sn->row_budget, bytes);
                atomic_store_explicit(&sn->blocks[s], row, memory_order_release);
            } else {
                free(row);
                row = NULL;
            }
        }
        pthread_mutex_unlock(&sn->row_mu);
    }
    if (row) {
        *lat = row[t];
        *rel = row[(size_t)A + t];
        return;
    }
    if (spe_table_get_latrel(sn->table, s, t, lat, rel) == SPE_OK) {
        if (atomic_load_explicit(&sn->host_reads, memory_order_relaxed) < 0) {   /* decided by that read */
            spe_table_layout l;
            memset(&l, 0, sizeof l);
            l.struct_size = sizeof l;
            if (spe_table_layout_get(sn->table, &l) == SPE_OK) atomic_store(&sn->host_reads, l.host_reads);
        }
        return;
    }
    spe_entry e;
    if (spe_table_get(sn->table, s, t, &e) == SPE_OK) {
        *lat = e.latency;
        *rel = e.reliability;
    } else {
        tlog(top, LOG_CRITICAL, "path table read failed: %s", spe_last_error());
        *lat = *rel = -1.0;
    }
}

/* ------------------------------------------------------ path cache model
 *
 * The reference caches a Path per ORDERED vertex pair (x, y) and answers a
 * query (s, t) with entry (s, t), else -- undirected graphs -- (t, s); on a miss
 * it stores entries and looks up (s, t), then (t, s) whatever the direction
 * (_topology_getPathEntry, shd-topology.c:1952-2034).  Stores
 * (_topology_shouldStorePath :1292-1321) never overwrite either direction of a
 * pair and keep non-direct paths out of complete graphs and off adjacent pairs
 * of prefer-direct graphs.  What a miss stores:
 *   DIRECT regime (complete, or preferdirectpaths and an s -> t edge): the
 *     single entry (s, t) (_topology_lookupDirectPath :1862-1912);
 *   s == t otherwise: the SELF entry (s, s) (:1530-1638);
 *   else s's Dijkstra row: (s, y) for every attached y (:1640-1860).
 * The model keeps explicit DIRECT / SELF entries in the shard maps and a row run
 * as one sequence number per source (run_seq), from which "was (x, y) stored by
 * x's row" follows: the row ran, the pair is storable, and neither direction
 * was stored before it.  The graph is one strong component, so every x != y
 * path exists; the row's own [x] path needs x's self-loop (quirk B5). */

static Shard* shard_of(Topology* top, uint64_t key) {
    return &top->shards[(key * 0x9E3779B97F4A7C15ull) >> 58];
}

/* the record of (x, y) in its locked shard, inserted when `insert` */
static PairRec* rec_locked(Shard* sh, uint64_t key, int insert) {
    if (insert && (sh->size + 1) * 2 > sh->cap) {
        const size_t nc = sh->cap ? sh->cap * 2 : 256;
        PairRec* nt = calloc(nc, sizeof(PairRec));
        for (size_t i = 0; i < sh->cap; ++i)
            if (sh->tab[i].key) {
                size_t j = (size_t)mix64(sh->tab[i].key) & (nc - 1);
                while (nt[j].key) j = (j + 1) & (nc - 1);
                nt[j] = sh->tab[i];
            }
        free(sh->tab);
        sh->tab = nt;
        sh->cap = nc;
    }
    if (!sh->cap) return NULL;
    size_t j = (size_t)mix64(key) & (sh->cap - 1);
    while (sh->tab[j].key) {
        if (sh->tab[j].key == key) return &sh->tab[j];
        j = (j + 1) & (sh->cap - 1);
    }
    if (!insert) return NULL;
    sh->tab[j].key = key;
    sh->size++;
    return &sh->tab[j];
}

static uint64_t pair_key(int32_t x, int32_t y) { return (((uint64_t)(uint32_t)x << 32) | (uint32_t)y) + 1; }

/* explicit entry (x, y): its store sequence (0 = none) and kind */
static uint64_t explicit_seq(Topology* top, int32_t x, int32_t y, int32_t* kind) {
    if (atomic_load_explicit(&top->n_explicit, memory_order_acquire) == 0) return 0;
    if (!atomic_load_explicit(&top->xflag[x], memory_order_acquire)) {
        if (kind) *kind = K_NONE;
        return 0;
    }
    const uint64_t key = pair_key(x, y);
    Shard* sh = shard_of(top, key);
    pthread_mutex_lock(&sh->mu);
    const PairRec* r = rec_locked(sh, key, 0);
    const uint64_t s = r ? r->seq : 0;
    if (kind) *kind = r ? r->kind : K_NONE;
    pthread_mutex_unlock(&sh->mu);
    return s;
}

static void explicit_store(Topology* top, int32_t x, int32_t y, int32_t kind, uint64_t seq) {
    const uint64_t key = pair_key(x, y);
    Shard* sh = shard_of(top, key);
    atomic_store_explicit(&top->xflag[x], 1, memory_order_release);   /* (before the entry is visible) */
    pthread_mutex_lock(&sh->mu);
    PairRec* r = rec_locked(sh, key, 1);
    if (!r->seq) {
        r->seq = seq;
        r->kind = kind;
        atomic_fetch_add_explicit(&top->n_explicit, 1, memory_order_release);
    }
    pthread_mutex_unlock(&sh->mu);
}

static uint64_t pair_count(Topology* top, int32_t x, int32_t y, uint64_t add) {
    const uint64_t key = pair_key(x, y);
    Shard* sh = shard_of(top, key);
    pthread_mutex_lock(&sh->mu);
    PairRec* r = rec_locked(sh, key, add != 0);
    uint64_t c = 0;
    if (r) c = (r->count += add);
    pthread_mutex_unlock(&sh->mu);
    return c;
}

static int adjacent(Topology* top, int32_t x, int32_t y) {
    int32_t a = 0;
    return spe_graph_adjacent(top->graph, x, y, &a) == SPE_OK && a;
}

static int direct_regime(Topology* top, int32_t s, int32_t t) {   /* :2002 */
    return top->complete || (top->prefer_direct && adjacent(top, s, t));
}

/* would x's Dijkstra row, run at sequence rx, store entry (x, y)?  `other` is
 * the run sequence of y's row (0 = none, or ignored when not earlier). */
static int row_stores(Topology* top, int32_t x, int32_t y, uint64_t rx, uint64_t ry) {
    if (top->complete) return 0;                                /* complete && !direct */
    if (top->prefer_direct && adjacent(top, x, y)) return 0;    /* a direct path exists */
    if (x == y) return adjacent(top, x, x);                     /* the [x] path needs the self-loop */
    int32_t k;
    const uint64_t ex = explicit_seq(top, x, y, &k), ey = explicit_seq(top, y, x, &k);
    if ((ex && ex < rx) || (ey && ey < rx)) return 0;           /* a direction already cached */
    if (ry && ry < rx && row_stores(top, y, x, ry, 0)) return 0;
    return 1;
}

/* store sequence of entry (x, y), 0 = not in the cache; *kind = K_DIRECT /
 * K_SELF for an explicit entry, K_NONE for a row entry */
static uint64_t entry_seq(Topology* top, int32_t x, int32_t y, int32_t* kind) {
    int32_t k = K_NONE;
    const uint64_t e = explicit_seq(top, x, y, &k);
    if (e) {
        if (kind) *kind = k;
        return e;
    }
    if (kind) *kind = K_NONE;
    const uint64_t rx = atomic_load_explicit(&top->run_seq[x], memory_order_acquire);
    if (!rx) return 0;
    const uint64_t ry = x == y ? 0 : atomic_load_explicit(&top->run_seq[y], memory_order_acquire);
    return row_stores(top, x, y, rx, ry) ? rx : 0;
}

static int find_entry(Topology* top, int32_t s, int32_t t, int reverse, int32_t* x, int32_t* y, int32_t* kind) {
    if (entry_seq(top, s, t, kind)) {
        *x = s;
        *y = t;
        return 1;
    }
    if (reverse && entry_seq(top, t, s, kind)) {
        *x = t;
        *y = s;
        return 1;
    }
    return 0;
}

static void note_min(Topology* top, double lat, int* updated) {   /* minimumPathLatency, :1359-1367 */
    if (!(lat > 0)) return;
    uint64_t cur = atomic_load(&top->stored_min_bits);
    uint64_t bits;
    memcpy(&bits, &lat, sizeof bits);
    while (cur == 0 || bits < cur) {   /* positive doubles order as integers */
        if (atomic_compare_exchange_weak(&top->stored_min_bits, &cur, bits)) {
            *updated = 1;
            break;
        }
    }
}

/* growable text for the path strings of log_row */
typedef struct {
    char* p;
    size_t len, cap;
} Buf;
static void buf_printf(Buf* b, const char* fmt, ...) {
    for (;;) {
        va_list ap;
        va_start(ap, fmt);
        const int k = vsnprintf(b->p ? b->p + b->len : NULL, b->p ? b->cap - b->len : 0, fmt, ap);
        va_end(ap);
        if (k < 0) return;
        if (b->p && b->len + (size_t)k < b->cap) {
            b->len += (size_t)k;
            return;
        }
        const size_t want = (b->cap ? b->cap : 256) * 2 + (size_t)k;
        char* q = realloc(b->p, want);
        if (!q) return;
        b->p = q;
        b->cap = want;
    }
}

/* The per-path lines of _topology_computeSourcePaths (:1809-1829): info for
 * the requested target, debug for the others, with the reference's path string
 * (:1413-1493): the source id, then "<--[latency,loss]-->id" per edge of the
 * get_eid edges along the row's path ("--[...]-->" when directed).  The path is
 * the parent walk of the row's shortest-path tree (spe_table_source_tree: the
 * source's rows are recomputed once, only when info lines are enabled). */
static void log_row(Topology* top, Snap* sn, int32_t s, int32_t want) {
    if (!log_on(top, LOG_INFO)) return;
    const int32_t ss = sn->slot_of_vertex[s];
    const int32_t n = top->n;
    int32_t* par = malloc(sizeof(int32_t) * (size_t)n);
    int32_t* vs = malloc(sizeof(int32_t) * ((size_t)n + 1));
    if (par && spe_table_source_tree(sn->table, ss, par) != SPE_OK) {
        free(par);
        par = NULL;
    }
    Buf b = {NULL, 0, 0};
    const char* arrow = top->directed ? "-->" : "<-->";
    for (int32_t j = 0; j < sn->A; ++j) {
        const int32_t t = sn->attached[j];
        const int lvl = t == want ? LOG_INFO : LOG_DEBUG;
        if (!log_on(top, lvl)) continue;
        spe_entry e;
        if (spe_table_get(sn->table, ss, j, &e) != SPE_OK || e.latency <= -1.0) continue;
        b.len = 0;
        buf_printf(&b, "%s", top->vstr[VS_ID][s]);
        int32_t nv = 0;
        if (par && vs) {   /* the path's vertices after the source ([s] for t == s: its self-loop) */
            for (int32_t x = t; x != s && x >= 0 && nv < n; x = par[x]) vs[nv++] = x;
            if (t == s) vs[nv++] = s;
            for (int32_t i = 0; i < nv / 2; ++i) {
                const int32_t tmp = vs[i];
                vs[i] = vs[nv - 1 - i];
                vs[nv - 1 - i] = tmp;
            }
        }
        int ok = 1;
        for (int32_t i = 0, from = s; i < nv && ok; ++i) {
            double w = 0.0, r = 0.0;
            ok = spe_graph_edge(top->graph, from, vs[i], &w, &r) == SPE_OK;   /* (s,s) needs its self-loop */
            buf_printf(&b, "%s[%f,%f]-->%s", top->directed ? "--" : "<--", w, 1.0f - r, top->vstr[VS_ID][vs[i]]);
            from = vs[i];
        }
        if (!ok) continue;
        tlog(top, lvl, "shortest path %s%s%s (%d%s%d) is %f ms with %f loss, path: %s", top->vstr[VS_ID][s], arrow,
             top->vstr[VS_ID][t], s, arrow, t, e.latency, 1 - e.reliability, b.p ? b.p : "");
    }
    free(b.p);
    free(vs);
    free(par);
}

/* _topology_getPathEntry on the model: the cached entry (x, y) answering (s, t);
 * stores on a miss.  Returns 0 when the reference's lookup finds no path. */
static int cache_lookup(Topology* top, Snap* sn, int32_t s, int32_t t, int32_t* x, int32_t* y, int32_t* kind,
                        int* min_updated) {
    if (find_entry(top, s, t, !top->directed, x, y, kind)) return 1;
    pthread_mutex_lock(&top->cache_mu);
    int found = find_entry(top, s, t, !top->directed, x, y, kind);
    int success = 1;
    if (!found) {
        const int ref = top->cache_mode == TOPOLOGY_ANSWER_REFERENCE;
        if (direct_regime(top, s, t)) {
            success = adjacent(top, s, t);   /* get_eid(s, t) must find the edge */
            if (success && !entry_seq(top, s, t, NULL) && !entry_seq(top, t, s, NULL)) {
                explicit_store(top, s, t, K_DIRECT, atomic_fetch_add(&top->seq, 1) + 1);
                if (ref) {
                    double l, r;
                    snap_value(top, sn, sn->slot_of_vertex[s], sn->slot_of_vertex[t], &l, &r);
                    note_min(top, l, min_updated);
                }
            }
        } else if (s == t) {
            spe_entry e;
            success = spe_graph_self_path(top->graph, s, &e) == SPE_OK && e.hops > 0;
            if (success && !entry_seq(top, s, s, NULL)) {
                explicit_store(top, s, s, K_SELF, atomic_fetch_add(&top->seq, 1) + 1);
                top->self_paths++;
                if (ref) note_min(top, e.latency, min_updated);
            }
        } else {
            /* the row run stores what it may; a re-run (directed graphs) stores nothing new */
            if (!atomic_load(&top->run_seq[s])) {
                const uint64_t rs = atomic_fetch_add(&top->seq, 1) + 1;
                atomic_store_explicit(&top->run_seq[s], rs, memory_order_release);
                log_row(top, sn, s, t);
                if (ref) {
                    const int32_t ss = sn->slot_of_vertex[s];
                    for (int32_t j = 0; j < sn->A; ++j)
                        if (entry_seq(top, s, sn->attached[j], NULL) == rs) {
                            double l, r;
                            snap_value(top, sn, ss, j, &l, &r);
                            note_min(top, l, min_updated);
                        }
                }
            }
            success = adjacent(top, s, s);   /* quirk B5: the row's [s] path fails without a self-loop */
        }
        if (success) found = find_entry(top, s, t, 1, x, y, kind);
    }
    pthread_mutex_unlock(&top->cache_mu);
    return found;
}

/* One query: resolve both addresses, publish a table that holds them if none
 * does yet, run the cache model, read the answer.  count_add > 0 increments the
 * packet counter of the answering entry (topology_incrementPathPacketCounter). */
static int query(Topology* top, uint32_t src, uint32_t dst, uint64_t count_add, double* lat, double* rel,
                 uint64_t* count_out) {
    *lat = *rel = -1.0;
    if (!top) return 0;
    for (int attempt = 0; attempt < 64; ++attempt) {   /* hosts may keep attaching meanwhile */
        state_rdlock(top);
        const int32_t sv = ip_get(top, src), dv = ip_get(top, dst);
        if (sv < 0 || dv < 0) {
            state_rdunlock(top);
            struct in_addr a = {sv < 0 ? src : dst};
            tlog(top, LOG_CRITICAL, "invalid vertex, %s address %s is not connected to topology",
                 sv < 0 ? "source" : "destination", inet_ntoa(a));
            return 0;
        }
        Snap* sn = top->snap;
        if (sn && sn->slot_of_vertex[sv] >= 0 && sn->slot_of_vertex[dv] >= 0) {
            int32_t x, y, kind = K_NONE;
            int min_updated = 0;
            const int found = cache_lookup(top, sn, sv, dv, &x, &y, &kind, &min_updated);
            int ok = 1;
            if (top->cache_mode == TOPOLOGY_ANSWER_REFERENCE) {
                if (!found) {
                    ok = 0;
                } else if (kind == K_SELF) {
                    spe_entry e;
                    spe_graph_self_path(top->graph, x, &e);
                    *lat = e.latency;
                    *rel = e.reliability;
                } else {
                    snap_value(top, sn, sn->slot_of_vertex[x], sn->slot_of_vertex[y], lat, rel);
                }
            } else {
                snap_value(top, sn, sn->slot_of_vertex[sv], sn->slot_of_vertex[dv], lat, rel);
            }
            if (found && (count_add || count_out)) {
                const uint64_t c = pair_count(top, x, y, count_add);
                if (count_out) *count_out = c;
            }
            state_rdunlock(top);
            if (!found && top->cache_mode == TOPOLOGY_ANSWER_REFERENCE) {   /* :2023-2029 */
                tlog(top, LOG_ERROR, "unable to find path between vertex %d (%s) and vertex %d (%s)", sv,
                     top->vstr[VS_ID][sv], dv, top->vstr[VS_ID][dv]);
            }
            if (min_updated && top->minlat_fn) {   /* worker_updateMinTimeJump, :1369 */
                double m;
                const uint64_t b = atomic_load(&top->stored_min_bits);
                memcpy(&m, &b, sizeof m);
                top->minlat_fn(m, top->minlat_ctx);
            }
            return ok && *lat > -1.0;
        }
        state_rdunlock(top);
        if (topology_seal(top) != SPE_OK) return 0;
    }
    return 0;
}

double topology_getLatency(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress) {
    double l, r;
    query(top, srcAddress, dstAddress, 0, &l, &r, NULL);
    return l;
}

double topology_getReliability(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress) {
    double l, r;
    query(top, srcAddress, dstAddress, 0, &l, &r, NULL);
    return r;
}

int32_t topology_getPathInfo(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress, double* latency,
                             double* reliability) {
    double l, r;
    const int ok = query(top, srcAddress, dstAddress, 0, &l, &r, NULL);
    if (latency) *latency = l;
    if (reliability) *reliability = r;
    return ok;
}

int32_t topology_isRoutable(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress) {
    return topology_getLatency(top, srcAddress, dstAddress) > -1 ? 1 : 0;   /* :2072-2075 */
}

void topology_incrementPathPacketCounter(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress) {
    double l, r;
    query(top, srcAddress, dstAddress, 1, &l, &r, NULL);   /* path->packetCount++, shd-path.c:53-56 */
}

/* Batches (worker_sendPacket's lookups for a whole round of packets).
 *
 * Phase 1, in parallel (up to SHADOW_SPE_BATCH_THREADS threads, default 16, for
 * batches of 64k queries and more), under the state lock shared: both addresses of
 * every query resolved, the published table checked to hold them (else the lock
 * is dropped, a covering table sealed and the phase redone), and the cache entry
 * answering each query looked up read-only (find_entry).  Phase 2, in query
 * order on the calling thread: every query phase 1 found no entry for runs the
 * full cache model (cache_lookup, which may store).  The model only ever adds
 * entries, first writer wins, and an entry found stays the one found: a store
 * made by an earlier query of the batch can turn a later miss into a hit but never
 * change a hit -- so the batch answers, counts and stores exactly as the same
 * queries made one by one in order would (tests/test_topology_batch.py).  Then
 * every table read of the batch at once: from the host mirror, or one device
 * lookup launch for the lot (spe_lookup_batch_host). */
enum { BQ_BAD = 0, BQ_HIT = 1, BQ_MISS = 2 };

typedef struct {
    Topology* top;
    Snap* sn;
    const spe_in_addr_t* src;
    const spe_in_addr_t* dst;
    int64_t a, b;
    int32_t* sv;   /* resolved vertices (-1: unknown address) */
    int32_t* dv;
    int32_t* x;    /* the answering entry (x, y) of a hit */
    int32_t* y;
    uint8_t* st;   /* BQ_* */
    int8_t* kind;
    int uncovered;
    /* the gather / finish passes */
    int32_t* pairs;
    const double* lat;
    uint8_t* routable;
    int64_t count;
    int resolve_only;   /* phase 1 without the cache entries (batch_entries does them) */
} BatchJob;

static void* batch_entries(void* p);

static void* batch_phase1(void* p) {
    BatchJob* j = p;
    Topology* top = j->top;
    Snap* sn = j->sn;
    for (int64_t i = j->a; i < j->b; ++i) {
        const int32_t sv = ip_get(top, j->src[i]), dv = ip_get(top, j->dst[i]);
        j->sv[i] = sv;
        j->dv[i] = dv;
        if (sv < 0 || dv < 0) {
            j->st[i] = BQ_BAD;
            continue;
        }
        if (sn->slot_of_vertex[sv] < 0 || sn->slot_of_vertex[dv] < 0) {
            j->uncovered = 1;
            return NULL;
        }
        j->st[i] = BQ_MISS;
    }
    return j->resolve_only ? NULL : batch_entries(p);
}

/* the answering cache entry of every resolved query (read-only: hits) */
static void* batch_entries(void* p) {
    BatchJob* j = p;
    Topology* top = j->top;
    for (int64_t i = j->a; i < j->b; ++i) {
        if (j->st[i] == BQ_BAD) continue;
        const int32_t sv = j->sv[i], dv = j->dv[i];
        int32_t x, y, kind = K_NONE;
        if (find_entry(top, sv, dv, !top->directed, &x, &y, &kind)) {
            j->st[i] = BQ_HIT;
            j->x[i] = x;
            j->y[i] = y;
            j->kind[i] = (int8_t)kind;
        } else {
            j->st[i] = BQ_MISS;
        }
    }
    return NULL;
}

/* default answer mode, device reads: query i reads slot pair i (bad addresses -1) */
static void* batch_gather(void* p) {
    BatchJob* j = p;
    const Snap* sn = j->sn;
    for (int64_t i = j->a; i < j->b; ++i) {
        const int bad = j->st[i] == BQ_BAD;
        j->pairs[2 * i] = bad ? -1 : sn->slot_of_vertex[j->sv[i]];
        j->pairs[2 * i + 1] = bad ? -1 : sn->slot_of_vertex[j->dv[i]];
        j->count += bad;
    }
    return NULL;
}

static void* batch_count(void* p) {   /* packet counts of the hits (they commute: any order) */
    BatchJob* j = p;
    for (int64_t i = j->a; i < j->b; ++i)
        if (j->st[i] == BQ_HIT) pair_count(j->top, j->x[i], j->y[i], 1);
    return NULL;
}

static void* batch_finish(void* p) {
    BatchJob* j = p;
    for (int64_t i = j->a; i < j->b; ++i) {
        j->routable[i] = j->lat[i] > -1.0;
        j->count += j->routable[i];
    }
    return NULL;
}

/* jobs[0 .. T) of one pass: jobs[1 ..] on their own threads, jobs[0] on this one */
static void batch_run(int T, BatchJob* jobs, void* (*fn)(void*)) {
    pthread_t th[64];
    int created[64] = {0};
    for (int k = 1; k < T; ++k) created[k] = pthread_create(&th[k], NULL, fn, &jobs[k]) == 0;
    fn(&jobs[0]);
    for (int k = 1; k < T; ++k) {
        if (created[k]) pthread_join(th[k], NULL);
        else fn(&jobs[k]);   /* no thread: this one does the share */
    }
}

/* the CPUs this process may use: its affinity mask, within a cgroup CPU quota if one is set */
static int host_cpus(void) {
    static int cached = 0;
    if (cached > 0) return cached;
    int n = 0;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (n <= 0) n = (int)sysconf(_SC_NPROCESSORS_ONLN);
    FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char q[32] = {0};
        long per = 0;
        if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
            const int quota = (int)((atol(q) + per - 1) / per);
            if (quota > 0 && quota < n) n = quota;
        }
        fclose(f);
    }
    cached = n > 0 ? n : 1;
    return cached;
}

static int batch_threads(int64_t n) {
    if (n < 65536) return 1;
    int t = host_cpus();   /* every CPU the process has (SHADOW_SPE_BATCH_THREADS overrides) */
    const char* e = getenv("SHADOW_SPE_BATCH_THREADS");
    if (e && atoi(e) > 0) t = atoi(e);
    if ((int64_t)t > n / 16384) t = (int)(n / 16384);
    return t < 1 ? 1 : (t > 64 ? 64 : t);
}

typedef struct {
    int32_t *sv, *dv, *x, *y;
    int32_t* pairs;   /* the device reads (slot pairs) and the query each answers */
    int64_t* at;
    uint8_t* st;
    int8_t* kind;
    void* mem;        /* one block for all the arrays */
    Topology* held;   /* the Topology whose cached scratch (batch_mu) this is, else NULL */
} BatchRes;

static void batch_res_free(BatchRes* r) {
    if (r->held) pthread_mutex_unlock(&r->held->batch_mu);
    else free(r->mem);
    memset(r, 0, sizeof *r);
}

/* 34 B per query in one block: the Topology's cached scratch when no other batch
 * holds it (already faulted in: a fresh 360-MB block per 20M-query batch spent
 * most of the batch in page faults, serialised across the threads), else a fresh one */
static int batch_res_alloc(Topology* top, int64_t n, BatchRes* r) {
    memset(r, 0, sizeof *r);
    const size_t bytes = (size_t)n * (6 * sizeof(int32_t) + sizeof(int64_t) + 2) + 64;
    if (pthread_mutex_trylock(&top->batch_mu) == 0) {
        if (top->bscr_bytes < bytes) {
            free(top->bscr);
            top->bscr = malloc(bytes);
            top->bscr_bytes = top->bscr ? bytes : 0;
            if (top->bscr) memset(top->bscr, 0, bytes);
        }
        if (top->bscr) {
            r->mem = top->bscr;
            r->held = top;
        } else {
            pthread_mutex_unlock(&top->batch_mu);
        }
    }
    if (!r->mem) r->mem = malloc(bytes);
    if (!r->mem) return 0;
    r->at = (int64_t*)r->mem;
    r->sv = (int32_t*)(r->at + n);
    r->dv = r->sv + n;
    r->x = r->dv + n;
    r->y = r->x + n;
    r->pairs = r->y + n;
    r->st = (uint8_t*)(r->pairs + 2 * n);
    r->kind = (int8_t*)(r->st + n);
    return 1;
}

/* Phase 1 (resolve_only: addresses only, the entries left to batch_entries).
 * Returns the snapshot with the state lock held shared, or NULL (lock released) when
 * no covering table could be sealed or memory ran out. */
static Snap* batch_prepare(Topology* top, int64_t n, const spe_in_addr_t* src, const spe_in_addr_t* dst, BatchRes* r,
                           int resolve_only) {
    if (!batch_res_alloc(top, n, r)) {
        batch_res_free(r);
        return NULL;
    }
    const int T = batch_threads(n);
    BatchJob jobs[64];
    for (int attempt = 0; attempt < 64; ++attempt) {
        state_rdlock(top);
        Snap* sn = top->snap;
        int covered = sn != NULL;
        if (covered) {
            for (int k = 0; k < T; ++k)
                jobs[k] = (BatchJob){top, sn, src, dst, n * k / T, n * (k + 1) / T,
                                     r->sv, r->dv, r->x, r->y, r->st, r->kind, 0, NULL, NULL, NULL, 0, resolve_only};
            batch_run(T, jobs, batch_phase1);
            for (int k = 0; k < T; ++k) covered &= !jobs[k].uncovered;
        }
        if (covered) return sn;
        state_rdunlock(top);
        if (topology_seal(top) != SPE_OK) break;
    }
    batch_res_free(r);
    return NULL;
}

static void batch_bad_address(Topology* top, int32_t sv, uint32_t src, uint32_t dst) {
    struct in_addr a = {sv < 0 ? src : dst};
    tlog(top, LOG_CRITICAL, "invalid vertex, %s address %s is not connected to topology",
         sv < 0 ? "source" : "destination", inet_ntoa(a));
}

static void batch_min_callback(Topology* top, int min_updated) {
    if (min_updated && top->minlat_fn) {   /* worker_updateMinTimeJump, :1369 */
        double m;
        const uint64_t b = atomic_load(&top->stored_min_bits);
        memcpy(&m, &b, sizeof m);
        top->minlat_fn(m, top->minlat_ctx);
    }
}

/* Phase 2: the misses in query order (stores happen here), bad addresses logged
 * in order; afterwards st[i] is BQ_HIT with (x, y, kind) or a failure. */
static void batch_phase2(Topology* top, Snap* sn, int64_t n, const spe_in_addr_t* src, const spe_in_addr_t* dst,
                         BatchRes* r, int* min_updated) {
    for (int64_t i = 0; i < n; ++i) {
        if (r->st[i] == BQ_BAD) {
            batch_bad_address(top, r->sv[i], src[i], dst[i]);
        } else if (r->st[i] == BQ_MISS) {
            int32_t x, y, kind = K_NONE;
            if (cache_lookup(top, sn, r->sv[i], r->dv[i], &x, &y, &kind, min_updated)) {
                r->st[i] = BQ_HIT;
                r->x[i] = x;
                r->y[i] = y;
                r->kind[i] = (int8_t)kind;
            }
        }
    }
}

typedef struct {
    const spe_table* table;
    const int32_t* pairs;
    int64_t n;
    double* lat;
    double* rel;
    uint8_t* ok;
    int rc;
    char err[256];   /* spe_last_error() is per thread: copied here on the thread that failed */
} LookupJob;

static void* batch_lookup(void* p) {   /* the device read of a batch, beside the cache bookkeeping */
    LookupJob* j = p;
    j->rc = spe_lookup_batch_host(j->table, j->pairs, j->n, j->lat, j->rel, j->ok);
    if (j->rc != SPE_OK) snprintf(j->err, sizeof(j->err), "%s", spe_last_error());
    return NULL;
}

int64_t topology_getPathInfoBatch(Topology* top, int64_t n, const spe_in_addr_t* srcAddress,
                                  const spe_in_addr_t* dstAddress, double* latency, double* reliability,
                                  uint8_t* routable) {
    if (!top || n < 0 || (n > 0 && (!srcAddress || !dstAddress || !latency || !reliability || !routable))) return -1;
    if (n == 0) return 0;
    const int timing = getenv("SHADOW_SPE_BATCH_TIMING") != NULL;
    const double t0 = timing ? now_s() : 0.0;
    const int ref = top->cache_mode == TOPOLOGY_ANSWER_REFERENCE;
    BatchRes r;
    /* rows mode: every query reads its own (s, t), so the table read can start as soon
     * as the addresses are resolved and run beside the path-cache bookkeeping */
    Snap* sn = batch_prepare(top, n, srcAddress, dstAddress, &r, !ref);
    if (!sn) {   /* no table could be sealed (or scratch failed): every query unanswered */
        for (int64_t i = 0; i < n; ++i) {
            latency[i] = -1.0;
            reliability[i] = -1.0;
            routable[i] = 0;
        }
        return -1;
    }
    const double t1 = timing ? now_s() : 0.0;
    /* (random reads of a whole-table host mirror cost ~100 ns each; one device launch
     * for a large batch costs ~25 B of PCIe traffic per query) */
    const int dev = n >= (sn->mlat ? 4096 : 256);
    int32_t* pairs = r.pairs;
    int64_t* at = r.at;
    int64_t nd = 0;
    const int T = batch_threads(n);
    BatchJob jobs[64];
    int min_updated = 0;
    double t2 = t1, t3 = t1;
    if (!ref) {
        LookupJob lj = {sn->table, pairs, n, latency, reliability, routable, SPE_OK, {0}};
        pthread_t lth;
        int lstarted = 0;
        if (dev) {   /* slot pairs (unknown addresses: -1, answered unroutable), then the read */
            for (int k = 0; k < T; ++k)
                jobs[k] = (BatchJob){top, sn, NULL, NULL, n * k / T, n * (k + 1) / T, r.sv, r.dv, NULL, NULL, r.st,
                                     NULL, 0, pairs, NULL, NULL, 0, 0};
            batch_run(T, jobs, batch_gather);
            lstarted = pthread_create(&lth, NULL, batch_lookup, &lj) == 0;
            if (!lstarted) batch_lookup(&lj);
        }
        for (int k = 0; k < T; ++k)   /* the cache entries of the hits (read-only) */
            jobs[k] = (BatchJob){top, sn, srcAddress, dstAddress, n * k / T, n * (k + 1) / T, r.sv, r.dv, r.x, r.y,
                                 r.st, r.kind, 0, NULL, NULL, NULL, 0, 0};
        batch_run(T, jobs, batch_entries);
        t2 = timing ? now_s() : 0.0;
        batch_phase2(top, sn, n, srcAddress, dstAddress, &r, &min_updated);
        t3 = timing ? now_s() : 0.0;
        if (lstarted) pthread_join(lth, NULL);
        if (!dev || lj.rc != SPE_OK) {
            if (dev) tlog(top, LOG_WARNING, "batched path table read failed (%s): reading per query", lj.err);
            for (int64_t i = 0; i < n; ++i) {
                latency[i] = reliability[i] = -1.0;
                if (r.st[i] == BQ_BAD) continue;
                snap_value(top, sn, sn->slot_of_vertex[r.sv[i]], sn->slot_of_vertex[r.dv[i]], &latency[i],
                           &reliability[i]);
            }
        }
    } else {   /* reference answers: the cached Path each query hits, after the misses in order */
        batch_phase2(top, sn, n, srcAddress, dstAddress, &r, &min_updated);
        t2 = t3 = timing ? now_s() : 0.0;
        for (int64_t i = 0; i < n; ++i) {
            latency[i] = reliability[i] = -1.0;
            if (r.st[i] == BQ_BAD) continue;
            if (r.st[i] != BQ_HIT) {   /* :2023-2029 */
                tlog(top, LOG_ERROR, "unable to find path between vertex %d (%s) and vertex %d (%s)", r.sv[i],
                     top->vstr[VS_ID][r.sv[i]], r.dv[i], top->vstr[VS_ID][r.dv[i]]);
                continue;
            }
            if (r.kind[i] == K_SELF) {
                spe_entry e;
                spe_graph_self_path(top->graph, r.x[i], &e);
                latency[i] = e.latency;
                reliability[i] = e.reliability;
                continue;
            }
            const int32_t s = sn->slot_of_vertex[r.x[i]], t = sn->slot_of_vertex[r.y[i]];
            if (dev) {
                pairs[2 * nd] = s;
                pairs[2 * nd + 1] = t;
                at[nd++] = i;
            } else {
                snap_value(top, sn, s, t, &latency[i], &reliability[i]);
            }
        }
        if (nd > 0) {
            double* lr = malloc((size_t)nd * 2 * sizeof(double));
            uint8_t* okd = malloc((size_t)nd);
            if (lr && okd && spe_lookup_batch_host(sn->table, pairs, nd, lr, lr + nd, okd) == SPE_OK) {
                for (int64_t k = 0; k < nd; ++k) {
                    latency[at[k]] = lr[k];
                    reliability[at[k]] = lr[nd + k];
                }
            } else {   /* per query */
                tlog(top, LOG_WARNING, "batched path table read failed (%s): reading per query", spe_last_error());
                for (int64_t k = 0; k < nd; ++k)
                    snap_value(top, sn, pairs[2 * k], pairs[2 * k + 1], &latency[at[k]], &reliability[at[k]]);
            }
            free(lr);
            free(okd);
        }
    }
    state_rdunlock(top);
    const double t4 = timing ? now_s() : 0.0;
    batch_res_free(&r);
    batch_min_callback(top, min_updated);
    for (int k = 0; k < T; ++k)
        jobs[k] = (BatchJob){top, NULL, NULL, NULL, n * k / T, n * (k + 1) / T, NULL, NULL, NULL, NULL, NULL, NULL,
                             0, NULL, latency, routable, 0, 0};
    batch_run(T, jobs, batch_finish);
    int64_t nok = 0;
    for (int k = 0; k < T; ++k) nok += jobs[k].count;
    if (timing)
        fprintf(stderr,
                "[topology] batch of %lld: resolve %.3f s, cached entries %.3f s, misses in order %.3f s, "
                "table reads (beside the two before, rows mode) done %.3f s later, finish %.3f s, total %.3f s\n",
                (long long)n, t1 - t0, t2 - t1, t3 - t2, t4 - t3, now_s() - t4, now_s() - t0);
    return nok;
}

void topology_incrementPathPacketCounterBatch(Topology* top, int64_t n, const spe_in_addr_t* srcAddress,
                                              const spe_in_addr_t* dstAddress) {
    if (!top || n <= 0 || !srcAddress || !dstAddress) return;
    BatchRes r;
    Snap* sn = batch_prepare(top, n, srcAddress, dstAddress, &r, 0);
    if (!sn) return;
    int min_updated = 0;
    batch_phase2(top, sn, n, srcAddress, dstAddress, &r, &min_updated);
    const int T = batch_threads(n);
    BatchJob jobs[64];
    for (int k = 0; k < T; ++k)
        jobs[k] = (BatchJob){top, sn, NULL, NULL, n * k / T, n * (k + 1) / T, NULL, NULL, r.x, r.y, r.st, NULL, 0,
                             NULL, NULL, NULL, 0, 0};
    batch_run(T, jobs, batch_count);
    state_rdunlock(top);
    batch_res_free(&r);
    batch_min_callback(top, min_updated);
}

uint64_t topology_path_packet_count(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress) {
    double l, r;
    uint64_t c = 0;
    query(top, srcAddress, dstAddress, 0, &l, &r, &c);
    return c;
}

double topology_min_path_latency(Topology* top) {
    if (!top || topology_seal(top) != SPE_OK) return 0.0;
    if (top->cache_mode == TOPOLOGY_ANSWER_REFERENCE) {
        double m = 0.0;
        const uint64_t b = atomic_load(&top->stored_min_bits);
        memcpy(&m, &b, sizeof m);
        return m;
    }
    state_rdlock(top);
    const double m = top->snap ? top->snap->min_latency : 0.0;
    state_rdunlock(top);
    return m;
}

/* _topology_logAllCachedPaths (:1914-1950) over the model: every explicit entry,
 * then every entry each source's row stored; path_toString's format
 * (shd-path.c:58-71). */
static void dump_entry(Topology* top, Snap* sn, int32_t x, int32_t y, int32_t kind, uint64_t count) {
    double l = -1.0, r = -1.0;
    if (kind == K_SELF) {
        spe_entry e;
        spe_graph_self_path(top->graph, x, &e);
        l = e.latency;
        r = e.reliability;
    } else if (sn && sn->slot_of_vertex[x] >= 0 && sn->slot_of_vertex[y] >= 0) {
        snap_value(top, sn, sn->slot_of_vertex[x], sn->slot_of_vertex[y], &l, &r);
    }
    tlog(top, LOG_INFO, "Found path %s%s%s in cache: SourceIndex=%d DestinationIndex=%d Latency=%f "
                        "Reliability=%f PacketCount=%llu isDirect=%s",
         top->vstr[VS_ID][x], top->directed ? "->" : "<->", top->vstr[VS_ID][y], x, y, l, r,
         (unsigned long long)count, kind == K_DIRECT ? "True" : "False");
}

int64_t topology_cached_path_count(Topology* top) {
    if (!top) return 0;
    int64_t n = atomic_load(&top->n_explicit);
    state_rdlock(top);
    Snap* sn = top->snap;
    for (int32_t x = 0; sn && x < top->n; ++x) {
        const uint64_t rx = atomic_load(&top->run_seq[x]);
        if (!rx) continue;
        for (int32_t j = 0; j < sn->A; ++j) {
            int32_t k;
            const int32_t y = sn->attached[j];
            if (!explicit_seq(top, x, y, &k) && entry_seq(top, x, y, NULL) == rx) ++n;
        }
    }
    state_rdunlock(top);
    return n;
}

void topology_free(Topology* top) {
    if (!top) return;
    if (log_on(top, LOG_INFO)) {
        Snap* sn = top->snap;
        for (int i = 0; i < NSHARD; ++i)
            for (size_t j = 0; j < top->shards[i].cap; ++j) {
                const PairRec* r = &top->shards[i].tab[j];
                if (!r->key || !r->seq) continue;
                dump_entry(top, sn, (int32_t)((r->key - 1) >> 32), (int32_t)((r->key - 1) & 0xffffffffu), r->kind,
                           r->count);
            }
        for (int32_t x = 0; sn && x < top->n; ++x) {
            const uint64_t rx = atomic_load(&top->run_seq[x]);
            if (!rx) continue;
            for (int32_t j = 0; j < sn->A; ++j) {
                int32_t k;
                const int32_t y = sn->attached[j];
                if (explicit_seq(top, x, y, &k) || entry_seq(top, x, y, NULL) != rx) continue;
                dump_entry(top, sn, x, y, K_NONE, pair_count(top, x, y, 0));
            }
        }
    }
    /* _topology_clearCache's timing line (:1262-1265); the rows are built on the GPU */
    tlog(top, LOG_MESSAGE, "path cache cleared, spent %f seconds computing %lld shortest paths with dijkstra, "
                           "and %f seconds computing %lld shortest self paths",
         top->build_seconds, (long long)top->build_rows, 0.0, (long long)top->self_paths);
    topo_release(top);
}
