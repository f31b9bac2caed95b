// mpi_bridge.cpp -- ComEx/ARMCI initialised over the caller's MPI communicator.
//
// Reference: comex_init_comm (comex/src-mpi-pr/comex.c:726-730) makes the
// communicator ComEx's world (_comex_init dups it); PARMCI_Init_mpi_comm
// (comex/src-armci/armci.c:427-440) calls it and returns 1 on success; GA's
// GA_Initialize_comm relies on it (global/src/base.c:545).  comex_group_comm
// (comex.h:78) hands out a group's communicator.
//
// libga_amd bootstraps without MPI (launcher hooks or the node-shm rendezvous),
// so it has no link dependency on an MPI library.  This file is compiled
// against MPICH's <mpi.h> -- the MPICH ABI (MPICH, Intel MPI, MVAPICH and Cray
// MPICH share MPI_Comm = int and the handle constants) -- and looks the MPI
// functions up in the process at the call (dlsym RTLD_DEFAULT): a program that
// hands us a communicator has MPI loaded.  The communicator's ranks become the
// bootstrap hooks' world (gaamd_set_bootstrap): its allgather and barrier are
// MPI_Allgather / MPI_Barrier on a dup of it, local ranks come from an
// allgather of host names.  A job on a sub-communicator therefore runs on that
// sub-communicator, not on MPI_COMM_WORLD.
#include <mpi.h>
#include <dlfcn.h>
#include <string.h>
#include <unistd.h>
#include <vector>
#include <map>
#include "runtime.hpp"
#include "../../include/comex.h"

namespace gaamd {
namespace {

struct Mpi {
    int (*initialized)(int *) = nullptr;
    int (*comm_dup)(MPI_Comm, MPI_Comm *) = nullptr;
    int (*comm_rank)(MPI_Comm, int *) = nullptr;
    int (*comm_size)(MPI_Comm, int *) = nullptr;
    int (*allgather)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm) = nullptr;
    int (*barrier)(MPI_Comm) = nullptr;
    int (*comm_group)(MPI_Comm, MPI_Group *) = nullptr;
    int (*group_incl)(MPI_Group, int, const int *, MPI_Group *) = nullptr;
    int (*comm_create_group)(MPI_Comm, MPI_Group, int, MPI_Comm *) = nullptr;
    int (*group_free)(MPI_Group *) = nullptr;
};

template <class F> void sym(F &f, const char *name) {
    f = reinterpret_cast<F>(dlsym(RTLD_DEFAULT, name));
    if (!f) fatal("%s: no MPI library in this process (comex_init_comm needs the caller's MPI, MPICH ABI)", name);
}

Mpi &mpi() {
    static Mpi m;
    static bool done = false;
    if (!done) {
        sym(m.initialized, "MPI_Initialized");
        sym(m.comm_dup, "MPI_Comm_dup");
        sym(m.comm_rank, "MPI_Comm_rank");
        sym(m.comm_size, "MPI_Comm_size");
        sym(m.allgather, "MPI_Allgather");
        sym(m.barrier, "MPI_Barrier");
        sym(m.comm_group, "MPI_Comm_group");
        sym(m.group_incl, "MPI_Group_incl");
        sym(m.comm_create_group, "MPI_Comm_create_group");
        sym(m.group_free, "MPI_Group_free");
        done = true;
    }
    return m;
}

MPI_Comm g_world = MPI_COMM_NULL;            // dup of the caller's communicator
std::map<int, MPI_Comm> g_group_comms;       // comex group -> its communicator (comex_group_comm)

int mpi_allgather(const void *send, void *recv, size_t bytes, void *) {
    // large payloads in pieces below 2^31 bytes per rank (the count is an int)
    const size_t piece = (size_t)1 << 30;
    int size = 0;
    mpi().comm_size(g_world, &size);
    if (bytes <= piece)
        return mpi().allgather(send, (int)bytes, MPI_BYTE, recv, (int)bytes, MPI_BYTE, g_world) == MPI_SUCCESS ? 0 : -1;
    std::vector<char> tmp(piece * (size_t)size);
    for (size_t off = 0; off < bytes; off += piece) {
        const size_t n = std::min(piece, bytes - off);
        if (mpi().allgather((const char *)send + off, (int)n, MPI_BYTE, tmp.data(), (int)n, MPI_BYTE, g_world) !=
            MPI_SUCCESS)
            return -1;
        for (int q = 0; q < size; ++q) memcpy((char *)recv + (size_t)q * bytes + off, tmp.data() + (size_t)q * n, n);
    }
    return 0;
}

int mpi_barrier(void *) { return mpi().barrier(g_world) == MPI_SUCCESS ? 0 : -1; }

}  // namespace

// hooks from a communicator: rank/size from it, local rank = position among the
// ranks with the same host name (the reference splits by host name too,
// comex/src-mpi-pr/groups.c:408-588)
static int bootstrap_from_comm(MPI_Comm comm) {
    Mpi &m = mpi();
    int inited = 0;
    m.initialized(&inited);
    if (!inited) fatal("comex_init_comm: MPI is not initialised");
    if (g_world == MPI_COMM_NULL && m.comm_dup(comm, &g_world) != MPI_SUCCESS)
        fatal("comex_init_comm: MPI_Comm_dup failed");
    int rank = 0, size = 1;
    m.comm_rank(g_world, &rank);
    m.comm_size(g_world, &size);
    char host[64];
    memset(host, 0, sizeof(host));
    gethostname(host, sizeof(host) - 1);
    if (const char *node = getenv("COMEX_AMD_NODE")) snprintf(host, sizeof(host), "node-%s", node);
    std::vector<char> all((size_t)size * sizeof(host));
    if (mpi_allgather(host, all.data(), sizeof(host), nullptr)) fatal("comex_init_comm: MPI_Allgather failed");
    int local = 0;
    for (int q = 0; q < rank; ++q)
        if (!memcmp(all.data() + (size_t)q * sizeof(host), host, sizeof(host))) ++local;
    return gaamd_set_bootstrap(rank, size, local, mpi_allgather, mpi_barrier, nullptr);
}

}  // namespace gaamd

using namespace gaamd;

extern "C" {

// the bootstrap half of comex_init_comm, without the GPU (tests: no device here)
int gaamd_set_bootstrap_comm(MPI_Comm comm) { return bootstrap_from_comm(comm); }

int comex_init_comm(MPI_Comm comm) {
    if (comex_initialized()) return COMEX_SUCCESS;   // _comex_init: initialised once
    if (!rt().boot_ready && bootstrap_from_comm(comm) != 0)
        fatal("comex_init_comm: the runtime already has another bootstrap");
    return comex_init();
}

// armci.c:427-440: 1 on success, 0 otherwise
int PARMCI_Init_mpi_comm(MPI_Comm comm) {
    extern int ARMCI_Default_Proc_Group;
    const int rc = comex_init_comm(comm);
    if (rc != COMEX_SUCCESS) return 0;
    ARMCI_Default_Proc_Group = 0;
    return 1;
}
int ARMCI_Init_mpi_comm(MPI_Comm comm) __attribute__((weak, alias("PARMCI_Init_mpi_comm")));

// comex.h:78: the group's communicator.  Only a runtime initialised over a
// communicator (comex_init_comm) has one; the world is the dup of it, another
// group a communicator over its members (created collectively over the group's
// members on the first call, as MPI_Comm_create_group requires, then kept).
int comex_group_comm(comex_group_t group, MPI_Comm *comm) {
    if (g_world == MPI_COMM_NULL)
        fatal("comex_group_comm(%d): the runtime was not initialised over a communicator (comex_init_comm); "
              "it bootstrapped without MPI and has none to hand out", group);
    if (group == COMEX_GROUP_WORLD) {
        *comm = g_world;
        return COMEX_SUCCESS;
    }
    auto it = g_group_comms.find(group);
    if (it == g_group_comms.end()) {
        const std::vector<int> members = group_members(group);
        MPI_Group wg, gg;
        MPI_Comm c = MPI_COMM_NULL;
        mpi().comm_group(g_world, &wg);
        mpi().group_incl(wg, (int)members.size(), members.data(), &gg);
        if (mpi().comm_create_group(g_world, gg, 0x6761 + group, &c) != MPI_SUCCESS)
            fatal("comex_group_comm(%d): MPI_Comm_create_group failed", group);
        mpi().group_free(&gg);
        mpi().group_free(&wg);
        it = g_group_comms.emplace(group, c).first;
    }
    *comm = it->second;
    return COMEX_SUCCESS;
}

// armci.h: ARMCI_Group is the comex group (armci.cpp)
MPI_Comm armci_group_comm(int *group) {
    MPI_Comm c = MPI_COMM_NULL;
    comex_group_comm(group && *group > 0 ? *group : COMEX_GROUP_WORLD, &c);
    return c;
}

}  // extern "C"
