"""The reference-side binding INTEGRATION.md §2 documents, compiled for real:
the adapter block is extracted from INTEGRATION.md and built against minimal
stand-in declarations of Shadow's types (gchar, Address, Random, the logger
and worker hooks -- the adapter's only dependencies), together with the shim
compiled the way a Shadow tree compiles it (-DSHD_TOPOLOGY_SPE_PREFIXED).  The
link must succeed with no duplicate and no unresolved topology symbol: the
reference-typed topology_* of shd-topology.h and the engine's spe_topology_*
coexist.  CPU only (nothing runs)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STANDIN = r"""
/* stand-in for Shadow's shadow.h: only what the adapter touches */
#include <stdint.h>
typedef char gchar;
typedef int gint;
typedef int gboolean;
typedef double gdouble;
typedef uint32_t guint32;
typedef uint64_t guint64;
typedef struct _Address Address;
typedef struct _Random Random;
guint32 address_toNetworkIP(Address* address);            /* shd-address.h:75 */
gdouble random_nextDouble(Random* random);                 /* shd-random.h:40 */
void worker_updateMinTimeJump(gdouble minPathLatency);     /* shd-worker.h:41 */
void error(const char* fmt, ...);
void critical(const char* fmt, ...);
void warning(const char* fmt, ...);
void message(const char* fmt, ...);
void info(const char* fmt, ...);
void debug(const char* fmt, ...);
/* shd-topology.h:12-25, the prototypes the adapter implements */
typedef struct _Topology Topology;
Topology* topology_new(const gchar* graphPath);
void topology_free(Topology* top);
void topology_attach(Topology* top, Address* address, Random* randomSourcePool, gchar* ipHint, gchar* citycodeHint,
                     gchar* countrycodeHint, gchar* geocodeHint, gchar* typeHint, guint64* bwDownOut,
                     guint64* bwUpOut);
void topology_detach(Topology* top, Address* address);
gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);
gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);
gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress);
"""

HOOKS = r"""
/* definitions of the stand-ins so the link is complete */
#include <stdarg.h>
#include "shadow.h"
guint32 address_toNetworkIP(Address* a) { return (guint32)(uintptr_t)a; }
gdouble random_nextDouble(Random* r) { (void)r; return 0.5; }
void worker_updateMinTimeJump(gdouble m) { (void)m; }
#define LOGF(name) void name(const char* fmt, ...) { (void)fmt; }
LOGF(error) LOGF(critical) LOGF(warning) LOGF(message) LOGF(info) LOGF(debug)
"""


def adapter_source():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. The adapter"):]
    return re.search(r"```c\n(.*?)```", sec, re.S).group(1)


def test_adapter_compiles_and_links_with_a_prefixed_shim(tmp_path):
    (tmp_path / "shadow.h").write_text(STANDIN)
    (tmp_path / "adapter.c").write_text(adapter_source())
    (tmp_path / "hooks.c").write_text(HOOKS)
    so = tmp_path / "libshadow_topology.so"
    cmd = ["gcc", "-std=c11", "-D_GNU_SOURCE", "-Wall", "-Werror", "-fPIC", "-shared", "-o", str(so),
           "-I", str(tmp_path), "-I", os.path.join(ROOT, "include"), "-I", "/usr/include/libxml2",
           str(tmp_path / "adapter.c"), str(tmp_path / "hooks.c"),
           "-DSHD_TOPOLOGY_SPE_PREFIXED", os.path.join(ROOT, "shadow_amd", "host", "shd_topology_spe.c"),
           "-L", os.path.join(ROOT, "shadow_amd"), "-lspe", "-lxml2", "-lpthread", "-lm", "-Wl,--no-undefined"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines()}
    for name in ("topology_new", "topology_free", "topology_attach", "topology_detach", "topology_isRoutable",
                 "topology_getLatency", "topology_getReliability", "topology_incrementPathPacketCounter"):
        assert name in syms and "spe_" + name in syms, name
