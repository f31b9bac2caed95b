// armci_msg.cpp -- the ARMCI message layer (include/message.h) on the MI355X
// runtime.
//
// Reference: comex/src-armci/message.c, where every call is an MPI collective or
// MPI_Send/Recv on the group's communicator.  This runtime bootstraps without
// MPI, so:
//   * point-to-point (armci_msg_snd/rcv/rcvany, message.c:354-463): tagged byte
//     messages over the job's socket transport (wire.cpp W_MSG frames), matched
//     by (sender, tag) in send order -- MPI's ordering guarantee;
//   * collectives over a group (gop, bcast, sel, barrier, message.c:188-757):
//     gathered to the group's first member by those messages, combined there in
//     member order (a deterministic order; MPI_Allreduce fixes none) and sent
//     back; the world barrier is the node-shm / launcher barrier of bootstrap.cpp.
// Semantics kept: the gop operators and types of armci_op_to_mpi_op /
// armci_type_to_mpi_type (message.c:54-124), abs for absmin/absmax (127-151),
// the comex_barrier before every gop and bcast (207, 233), sel by MINLOC/MAXLOC
// then a bcast of the winner's payload (255-324), the heap-shaped bintree
// (543-561), and the calls the reference leaves unimplemented fail the same way
// (clus_* and armci_grp_clus_brdcst, 616-650, 757).
#include "../../include/armci.h"
#include "../../include/message.h"
#include "../../include/comex.h"
#include "runtime.hpp"
#include <string.h>
#include <time.h>
#include <vector>

extern "C" int ARMCI_Default_Proc_Group;   // armci.cpp (groups.c:10)

namespace gaamd {

namespace {
// internal message tags (above any tag a GA build uses): kind + 16 * group key
constexpr int kTagBase = 0x40000000;
enum { T_GATHER = 0, T_RESULT = 1, T_BAR_IN = 2, T_BAR_OUT = 3, T_BCAST = 4 };
int tag_of(int key, int kind) { return kTagBase + (((key + 4) & 0x3ffff) << 4) + kind; }
constexpr int kGroupSelf = -2;   // message.c:20 ARMCI_GROUP_SELF

int my_index(const std::vector<int> &m) {
    const int me = rt().rank;
    for (size_t i = 0; i < m.size(); ++i)
        if (m[i] == me) return (int)i;
    fatal("armci_msg: rank %d is not a member of the group", me);
}

std::vector<int> members_of(int group) {
    if (group == kGroupSelf) return std::vector<int>(1, rt().rank);
    return group_members(group);
}

size_t type_size(int type) {
    switch (type) {
    case ARMCI_INT: return sizeof(int);
    case ARMCI_LONG: return sizeof(long);
    case ARMCI_LONG_LONG: return sizeof(long long);
    case ARMCI_FLOAT: return sizeof(float);
    case ARMCI_DOUBLE: return sizeof(double);
    }
    fatal("armci_msg: unsupported type %d", type);
}

// message.c:81-124: the operator, by prefix in the reference's order
enum Op { O_SUM, O_MAX, O_MIN, O_PROD, O_BOR, O_LAND, O_LOR, O_BAND };
Op parse_op(const char *op) {
    if (!strncmp(op, "+", 1)) return O_SUM;
    if (!strncmp(op, "max", 3)) return O_MAX;
    if (!strncmp(op, "min", 3)) return O_MIN;
    if (!strncmp(op, "*", 1)) return O_PROD;
    if (!strncmp(op, "absmin", 6)) return O_MIN;
    if (!strncmp(op, "absmax", 6)) return O_MAX;
    if (!strncmp(op, "or", 2)) return O_BOR;
    if (!strncmp(op, "&&", 2) || !strncmp(op, "land", 4)) return O_LAND;
    if (!strncmp(op, "||", 2) || !strncmp(op, "lor", 3)) return O_LOR;
    if (!strncmp(op, "&", 1) || !strncmp(op, "band", 4)) return O_BAND;
    if (!strncmp(op, "|", 1) || !strncmp(op, "bor", 3)) return O_BOR;
    fatal("Unsupported gop operation %s", op);
}

template <typename T> void combine_int(T *a, const T *b, int n, Op op) {
    for (int i = 0; i < n; ++i) {
        switch (op) {
        case O_SUM: a[i] = a[i] + b[i]; break;
        case O_PROD: a[i] = a[i] * b[i]; break;
        case O_MAX: a[i] = b[i] > a[i] ? b[i] : a[i]; break;
        case O_MIN: a[i] = b[i] < a[i] ? b[i] : a[i]; break;
        case O_BOR: a[i] = a[i] | b[i]; break;
        case O_BAND: a[i] = a[i] & b[i]; break;
        case O_LAND: a[i] = (a[i] && b[i]) ? 1 : 0; break;
        case O_LOR: a[i] = (a[i] || b[i]) ? 1 : 0; break;
        }
    }
}
template <typename T> void combine_flt(T *a, const T *b, int n, Op op) {
    for (int i = 0; i < n; ++i) {
        switch (op) {
        case O_SUM: a[i] = a[i] + b[i]; break;
        case O_PROD: a[i] = a[i] * b[i]; break;
        case O_MAX: a[i] = b[i] > a[i] ? b[i] : a[i]; break;
        case O_MIN: a[i] = b[i] < a[i] ? b[i] : a[i]; break;
        case O_LAND: a[i] = (a[i] != 0 && b[i] != 0) ? 1 : 0; break;
        case O_LOR: a[i] = (a[i] != 0 || b[i] != 0) ? 1 : 0; break;
        default: fatal("bitwise gop on a floating-point type");
        }
    }
}
void combine(void *a, const void *b, int n, int type, Op op) {
    switch (type) {
    case ARMCI_INT: combine_int((int *)a, (const int *)b, n, op); return;
    case ARMCI_LONG: combine_int((long *)a, (const long *)b, n, op); return;
    case ARMCI_LONG_LONG: combine_int((long long *)a, (const long long *)b, n, op); return;
    case ARMCI_FLOAT: combine_flt((float *)a, (const float *)b, n, op); return;
    case ARMCI_DOUBLE: combine_flt((double *)a, (const double *)b, n, op); return;
    }
    fatal("armci_msg: unsupported type %d", type);
}

// message.c:127-151
void do_abs(void *x, int n, int type) {
#define GA_ABS(T)                                                  \
    {                                                              \
        T *y = (T *)x;                                             \
        for (int i = 0; i < n; ++i) y[i] = y[i] >= 0 ? y[i] : -y[i]; \
        return;                                                    \
    }
    switch (type) {
    case ARMCI_INT: GA_ABS(int)
    case ARMCI_LONG: GA_ABS(long)
    case ARMCI_LONG_LONG: GA_ABS(long long)
    case ARMCI_FLOAT: GA_ABS(float)
    case ARMCI_DOUBLE: GA_ABS(double)
    }
#undef GA_ABS
    fatal("unsupported ABS operation");
}

// the barrier of a group before its gop/bcast (comex_barrier(group), message.c:207)
void group_fence_barrier(int group) {
    if (group == kGroupSelf) return;
    comex_barrier(group);
}

// message.c:188-225: allreduce of x over the group
void do_gop(void *x, int n, const char *op, int type, int group) {
    const Op o = parse_op(op);
    if (!strncmp(op, "absmin", 6) || !strncmp(op, "absmax", 6)) do_abs(x, n, type);
    const std::vector<int> m = members_of(group);
    if (m.size() <= 1 || n <= 0) return;
    group_fence_barrier(group);
    const size_t bytes = (size_t)n * type_size(type);
    const int me = my_index(m);
    if (me == 0) {
        std::vector<char> in(bytes);
        for (size_t k = 1; k < m.size(); ++k) {
            msg_recv(m[k], tag_of(group, T_GATHER), in.data(), bytes, nullptr);
            combine(x, in.data(), n, type, o);
        }
        for (size_t k = 1; k < m.size(); ++k) msg_send(m[k], tag_of(group, T_RESULT), x, bytes);
    } else {
        msg_send(m[0], tag_of(group, T_GATHER), x, bytes);
        msg_recv(m[0], tag_of(group, T_RESULT), x, bytes, nullptr);
    }
}

int default_group() { return ARMCI_Default_Proc_Group; }

// the node group of armci_init_domains (armci.c:88-95): ranks of this node, or self
int node_group_members_key(std::vector<int> &m) {
    Runtime &r = rt();
    m.clear();
    for (int q = 0; q < r.size; ++q)
        if (r.same_node(q)) m.push_back(q);
    return -3;   // a key of its own
}

void do_gop_members(void *x, int n, const char *op, int type, const std::vector<int> &m, int key) {
    const Op o = parse_op(op);
    if (!strncmp(op, "absmin", 6) || !strncmp(op, "absmax", 6)) do_abs(x, n, type);
    if (m.size() <= 1 || n <= 0) return;
    members_barrier(m, key);
    const size_t bytes = (size_t)n * type_size(type);
    const int me = my_index(m);
    if (me == 0) {
        std::vector<char> in(bytes);
        for (size_t k = 1; k < m.size(); ++k) {
            msg_recv(m[k], tag_of(key, T_GATHER), in.data(), bytes, nullptr);
            combine(x, in.data(), n, type, o);
        }
        for (size_t k = 1; k < m.size(); ++k) msg_send(m[k], tag_of(key, T_RESULT), x, bytes);
    } else {
        msg_send(m[0], tag_of(key, T_GATHER), x, bytes);
        msg_recv(m[0], tag_of(key, T_RESULT), x, bytes, nullptr);
    }
}
}  // namespace

void members_barrier(const std::vector<int> &m, int key) {
    if (m.size() <= 1) return;
    Runtime &r = rt();
    if (m.size() == (size_t)r.size) {   // the whole job: the bootstrap barrier
        boot_barrier();
        return;
    }
    const int me = my_index(m);
    char t = 0;
    if (me == 0) {
        for (size_t k = 1; k < m.size(); ++k) msg_recv(m[k], tag_of(key, T_BAR_IN), &t, 1, nullptr);
        for (size_t k = 1; k < m.size(); ++k) msg_send(m[k], tag_of(key, T_BAR_OUT), &t, 1);
    } else {
        msg_send(m[0], tag_of(key, T_BAR_IN), &t, 1);
        msg_recv(m[0], tag_of(key, T_BAR_OUT), &t, 1, nullptr);
    }
}

void members_bcast(const std::vector<int> &m, int key, void *buf, size_t bytes, int root_index) {
    if (m.size() <= 1) return;
    const int me = my_index(m);
    if (me == root_index) {
        for (size_t k = 0; k < m.size(); ++k)
            if ((int)k != root_index) msg_send(m[k], tag_of(key, T_BCAST), buf, bytes);
    } else {
        msg_recv(m[root_index], tag_of(key, T_BCAST), buf, bytes, nullptr);
    }
}

void members_allgather(const std::vector<int> &m, int key, const void *send, void *recv, size_t bytes) {
    Runtime &r = rt();
    bool world_order = m.size() == (size_t)r.size;
    for (size_t k = 0; k < m.size() && world_order; ++k) world_order = m[k] == (int)k;
    if (world_order) {
        boot_allgather(send, recv, bytes);
        return;
    }
    const int me = my_index(m);
    char *out = (char *)recv;
    memcpy(out + (size_t)me * bytes, send, bytes);
    if (m.size() <= 1) return;
    if (me == 0) {
        for (size_t k = 1; k < m.size(); ++k) msg_recv(m[k], tag_of(key, T_GATHER), out + k * bytes, bytes, nullptr);
    } else {
        msg_send(m[0], tag_of(key, T_GATHER), send, bytes);
    }
    members_bcast(m, key, recv, bytes * m.size(), 0);
}

}  // namespace gaamd

using namespace gaamd;

extern "C" {

void armci_msg_snd(int tag, void *buffer, int len, int to) {
    if (len < 0) fatal("armci_msg_snd: negative length");
    msg_send(to, tag, buffer, (size_t)len);
}

void armci_msg_rcv(int tag, void *buffer, int len, int *msglen, int from) {
    const size_t n = msg_recv(from, tag, buffer, (size_t)(len < 0 ? 0 : len), nullptr);
    if (msglen) *msglen = (int)n;
}

int armci_msg_rcvany(int tag, void *buffer, int len, int *msglen) {
    int src = -1;
    const size_t n = msg_recv(-1, tag, buffer, (size_t)(len < 0 ? 0 : len), &src);
    if (msglen) *msglen = (int)n;
    return src;
}

void armci_msg_reduce(void *x, int n, char *op, int type) { do_gop(x, n, op, type, default_group()); }

void armci_msg_reduce_scope(int scope, void *x, int n, char *op, int type) {
    armci_msg_gop_scope(scope, x, n, op, type);
}

void armci_msg_gop_scope(int scope, void *x, int n, char *op, int type) {
    if (scope == SCOPE_NODE) {
        std::vector<int> m;
        const int key = node_group_members_key(m);
        do_gop_members(x, n, op, type, m, key);
    } else {
        do_gop(x, n, op, type, default_group());
    }
}

void armci_msg_igop(int *x, int n, char *op) { do_gop(x, n, op, ARMCI_INT, default_group()); }
void armci_msg_lgop(long *x, int n, char *op) { do_gop(x, n, op, ARMCI_LONG, default_group()); }
void armci_msg_llgop(long long *x, int n, char *op) { do_gop(x, n, op, ARMCI_LONG_LONG, default_group()); }
void armci_msg_fgop(float *x, int n, char *op) { do_gop(x, n, op, ARMCI_FLOAT, default_group()); }
void armci_msg_dgop(double *x, int n, char *op) { do_gop(x, n, op, ARMCI_DOUBLE, default_group()); }

// message.c:228-236: root is a rank of the default group
void armci_msg_bcast(void *buf, int len, int root) {
    if (!buf && len > 0) fatal("armci_msg_bcast: NULL buffer");
    comex_barrier(default_group());
    const std::vector<int> m = members_of(default_group());
    members_bcast(m, default_group(), buf, (size_t)len, root);
}

void armci_msg_brdcst(void *buffer, int len, int root) { armci_msg_bcast(buffer, len, root); }

void armci_msg_bcast_scope(int scope, void *buffer, int len, int root) {
    if (scope == SCOPE_ALL || scope == SCOPE_MASTERS) {
        armci_msg_bcast(buffer, len, root);
    } else if (scope == SCOPE_NODE) {
        std::vector<int> m;
        const int key = node_group_members_key(m);
        members_bcast(m, key, buffer, (size_t)len, root);
    } else {
        fatal("unsupported armci_msg_bcast_scope scope %d", scope);
    }
}

// message.c:255-324: the rank holding the min / max of the leading value wins (the
// lowest such rank, as MPI_MINLOC/MAXLOC), then its whole n-byte payload is
// broadcast; `contribute` is not used by the reference either
void armci_msg_sel_scope(int scope, void *x, int n, char *op, int type, int contribute) {
    (void)contribute;
    const bool mn = !strncmp(op, "min", 3);
    if (!mn && strncmp(op, "max", 3)) fatal("unsupported armci_msg_sel_scope operation %s", op);
    std::vector<int> m;
    int key;
    if (scope == SCOPE_NODE) {
        key = node_group_members_key(m);
    } else {
        comex_barrier(default_group());
        key = default_group();
        m = members_of(key);
    }
    const size_t ts = type_size(type);
    std::vector<char> vals(ts * m.size());
    members_allgather(m, key, x, vals.data(), ts);
    int win = 0;
    for (size_t k = 1; k < m.size(); ++k) {
        const char *a = vals.data() + (size_t)win * ts, *b = vals.data() + k * ts;
        bool better = false;
        switch (type) {
#define GA_SEL(T) { const T va = *(const T *)a, vb = *(const T *)b; better = mn ? vb < va : vb > va; break; }
        case ARMCI_INT: GA_SEL(int)
        case ARMCI_LONG: GA_SEL(long)
        case ARMCI_LONG_LONG: GA_SEL(long long)
        case ARMCI_FLOAT: GA_SEL(float)
        case ARMCI_DOUBLE: GA_SEL(double)
#undef GA_SEL
        default: fatal("unsupported SELECT operation");
        }
        if (better) win = (int)k;
    }
    members_bcast(m, key, x, (size_t)n, win);
}

void armci_exchange_address(void *ptr_ar[], int n) {
    int g = default_group();
    armci_exchange_address_grp(ptr_ar, n, &g);
}

// every member's ptr_arr[my group rank] to everybody (the reference's disabled
// MPI_Allgather, message.c:692-714, which it replaces with an error)
void armci_exchange_address_grp(void *ptr_arr[], int n, ARMCI_Group *group) {
    const std::vector<int> m = members_of(*group);
    if ((size_t)n < m.size()) fatal("armci_exchange_address_grp: %d entries for %zu ranks", n, m.size());
    const int me = my_index(m);
    std::vector<void *> all(m.size());
    members_allgather(m, *group, &ptr_arr[me], all.data(), sizeof(void *));
    for (size_t k = 0; k < m.size(); ++k) ptr_arr[k] = all[k];
}

void parmci_msg_barrier() {
    comex_barrier(default_group());
    members_barrier(members_of(default_group()), default_group());
}

void armci_msg_bintree(int scope, int *Root, int *Up, int *Left, int *Right) {
    if (scope == SCOPE_NODE || scope == SCOPE_MASTERS) fatal("armci_msg_bintree: scope %d", scope);
    const int root = 0, nproc = armci_msg_nproc(), index = armci_msg_me() - root;
    int up = (index - 1) / 2 + root;
    if (up < root) up = -1;
    int left = 2 * index + 1 + root;
    if (left >= root + nproc) left = -1;
    int right = 2 * index + 2 + root;
    if (right >= root + nproc) right = -1;
    *Up = up;
    *Left = left;
    *Right = right;
    *Root = root;
}

int armci_msg_me() {
    if (!comex_initialized()) fatal("armci_msg_me before ARMCI_Init");
    return rt().rank;
}

int armci_msg_nproc() {
    if (!comex_initialized()) fatal("armci_msg_nproc before ARMCI_Init");
    return rt().size;
}

void armci_msg_abort(int code) {
    fprintf(stderr, "Exiting, Error in Communication\n");
    fatal("armci_msg_abort(%d)", code);
}

// no MPI underneath: the launcher owns process start-up and tear-down
void armci_msg_init(int *argc, char ***argv) {
    (void)argc;
    (void)argv;
}
void armci_msg_finalize() {}

double armci_timer() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

void armci_msg_clus_brdcst(void *, int) { fatal("armci_msg_clus_brdcst not implemented"); }
void armci_msg_clus_igop(int *, int, char *) { fatal("armci_msg_clus_igop not implemented"); }
void armci_msg_clus_fgop(float *, int, char *) { fatal("armci_msg_clus_fgop not implemented"); }
void armci_msg_clus_lgop(long *, int, char *) { fatal("armci_msg_clus_lgop not implemented"); }
void armci_msg_clus_llgop(long long *, int, char *) { fatal("armci_msg_clus_llgop not implemented"); }
void armci_msg_clus_dgop(double *, int, char *) { fatal("armci_msg_clus_dgop not implemented"); }

void armci_msg_group_gop_scope(int scope, void *x, int n, char *op, int type, ARMCI_Group *group) {
    do_gop(x, n, op, type, scope == SCOPE_NODE ? kGroupSelf : *group);
}
void armci_msg_group_igop(int *x, int n, char *op, ARMCI_Group *group) { do_gop(x, n, op, ARMCI_INT, *group); }
void armci_msg_group_lgop(long *x, int n, char *op, ARMCI_Group *group) { do_gop(x, n, op, ARMCI_LONG, *group); }
void armci_msg_group_llgop(long long *x, int n, char *op, ARMCI_Group *group) {
    do_gop(x, n, op, ARMCI_LONG_LONG, *group);
}
void armci_msg_group_fgop(float *x, int n, char *op, ARMCI_Group *group) { do_gop(x, n, op, ARMCI_FLOAT, *group); }
void armci_msg_group_dgop(double *x, int n, char *op, ARMCI_Group *group) {
    do_gop(x, n, op, ARMCI_DOUBLE, *group);
}

void parmci_msg_group_barrier(ARMCI_Group *group) {
    comex_barrier(*group);
    members_barrier(members_of(*group), *group);
}

// message.c:724-755: `root` is a WORLD rank; the group's members receive its bytes
void armci_msg_group_bcast_scope(int scope, void *buf, int len, int root, ARMCI_Group *group) {
    if (scope == SCOPE_NODE) {
        std::vector<int> m;
        const int key = node_group_members_key(m);
        members_bcast(m, key, buf, (size_t)len, root);
        return;
    }
    const std::vector<int> m = members_of(*group);
    int root_sub = -1;
    for (size_t k = 0; k < m.size(); ++k)
        if (m[k] == root) root_sub = (int)k;
    if (root_sub < 0) fatal("armci_msg_group_bcast_scope: root %d is not in the group", root);
    comex_barrier(*group);
    members_bcast(m, *group, buf, (size_t)len, root_sub);
}

void armci_grp_clus_brdcst(void *, int, int, int, ARMCI_Group *) { fatal("armci_grp_clus_brdcst not implemented"); }

// capi.c:544-557: armci_msg_barrier / armci_msg_group_barrier are weak wrappers
void armci_msg_barrier() __attribute__((weak, alias("parmci_msg_barrier")));
void armci_msg_group_barrier(ARMCI_Group *) __attribute__((weak, alias("parmci_msg_group_barrier")));

}  // extern "C"
