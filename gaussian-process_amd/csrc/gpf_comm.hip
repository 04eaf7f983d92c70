// gpf_comm.hip — the swarm exchange behind the C-ABI.
//
// One process per GPU. After each batch of particle evaluations every rank needs the whole
// score vector, so that all ranks take the same first-index argmin for the global best
// (find_len_scales.py:81,110) and draw identical r1/r2 (:91-92). The reference has no such
// step: its single process fans the swarm out to a fork pool (:73-77,102-104,133-135).
// Here rank r scores rows [rP/G, (r+1)P/G) and one all-reduce (sum) of a zero-initialised
// [P + G] vector gives every rank the full scores: exact, since every score entry has exactly
// one non-zero contributor. The G trailing entries carry each rank's status (0 = ok,
// 1 + first non-PD particle, -code on a HIP error), so an error on one rank is raised on every
// rank instead of leaving the others blocked in the collective.
//
// Transports:
//   GPF_COMM_RCCL  ncclAllReduce (float64) on the context's device, over xGMI between the
//                  GPUs of one node; the ncclUniqueId is handed out by rank 0 over TCP.
//   GPF_COMM_HOST  the same exchange over the TCP sockets of the rendezvous (rank 0 sums the
//                  ranks' vectors in rank order and sends the result back): needs no device;
//                  the CPU tests use it to run the C exchange at 2..8 ranks.

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <thread>

struct gpf_comm {
  int rank = 0, nranks = 1, transport = GPF_COMM_HOST;
  int device = -1;
  std::vector<int> fd;  // rank 0: fd[r] = socket to rank r (fd[0] unused); others: fd[0] = socket to rank 0
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  double* d_buf = nullptr;
  double* h_buf = nullptr;  // pinned staging for the device all-reduce
  size_t cap = 0;
  int timeout_ms = 600000;
  std::string err;
  double xch_ms = 0.0;  // wall time inside gpf_comm_exchange_scores (gpf_comm_stats)
  long long xch_n = 0;
};

namespace {

int comm_fail(gpf_comm* c, const std::string& m, int code = GPF_HIP_ERROR) {
  c->err = m;
  return code;
}

// Blocking send/recv of exactly n bytes with an overall deadline (a dead peer must not hang
// the caller forever).
bool io_all(int fd, void* buf, size_t n, bool send, int timeout_ms) {
  char* p = static_cast<char*>(buf);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (n > 0) {
    const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(t_end - std::chrono::steady_clock::now()).count();
    if (left <= 0) return false;
    pollfd pf{fd, (short)(send ? POLLOUT : POLLIN), 0};
    const int pr = poll(&pf, 1, left);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    const ssize_t k = send ? ::send(fd, p, n, MSG_NOSIGNAL) : ::recv(fd, p, n, 0);
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool resolve(const char* host, int port, sockaddr_in& sa) {
  std::memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host, &sa.sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) return false;
  sa.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

void nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// Rendezvous: rank 0 listens on host:port and accepts nranks-1 peers (each announces its
// rank); the others connect (retrying until the deadline: rank 0 may start later).
int rendezvous(gpf_comm* c, const char* host, int port) {
  sockaddr_in sa;
  if (!resolve(host, port, sa)) return comm_fail(c, std::string("gpf_comm_open: cannot resolve ") + host, GPF_BAD_ARG);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(c->timeout_ms);
  auto left_ms = [&] {
    return (int)std::chrono::duration_cast<std::chrono::milliseconds>(t_end - std::chrono::steady_clock::now()).count();
  };
  if (c->rank == 0) {
    c->fd.assign(c->nranks, -1);
    const int ls = socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return comm_fail(c, "gpf_comm_open: socket failed");
    int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (bind(ls, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || listen(ls, c->nranks) != 0) {
      close(ls);
      return comm_fail(c, "gpf_comm_open: cannot listen on " + std::string(host) + ":" + std::to_string(port) + " (" +
                              strerror(errno) + ")");
    }
    for (int got = 1; got < c->nranks;) {
      pollfd pf{ls, POLLIN, 0};
      const int lm = left_ms();
      if (lm <= 0 || poll(&pf, 1, lm) <= 0) {
        close(ls);
        return comm_fail(c, "gpf_comm_open: timed out waiting for " + std::to_string(c->nranks - got) + " rank(s)");
      }
      const int fd = accept(ls, nullptr, nullptr);
      if (fd < 0) continue;
      int32_t r = -1;
      if (!io_all(fd, &r, 4, false, c->timeout_ms) || r <= 0 || r >= c->nranks || c->fd[r] >= 0) {
        close(fd);
        close(ls);
        return comm_fail(c, "gpf_comm_open: bad or duplicate rank announcement " + std::to_string(r));
      }
      nodelay(fd);
      c->fd[r] = fd;
      ++got;
    }
    close(ls);
  } else {
    c->fd.assign(1, -1);
    for (;;) {
      const int fd = socket(AF_INET, SOCK_STREAM, 0);
      if (fd < 0) return comm_fail(c, "gpf_comm_open: socket failed");
      if (connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
        nodelay(fd);
        c->fd[0] = fd;
        break;
      }
      close(fd);
      if (left_ms() <= 0) return comm_fail(c, "gpf_comm_open: cannot reach rank 0 at " + std::string(host) + ":" + std::to_string(port));
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    int32_t r = c->rank;
    if (!io_all(c->fd[0], &r, 4, true, c->timeout_ms)) return comm_fail(c, "gpf_comm_open: announcement failed");
  }
  return GPF_OK;
}

// Every rank's status word to every rank over the rendezvous sockets (star through rank 0): the
// ranks agree on each step of the RCCL bootstrap before the next, so a failure on one rank fails
// all of them at that step instead of leaving the others blocked in ncclCommInitRank or in the
// first all-reduce. Returns the number of ranks whose word was nonzero, or -1 on a socket error.
int host_agree(gpf_comm* c, int32_t mine) {
  int32_t bad = mine != 0;
  if (c->nranks == 1) return bad;
  if (c->rank == 0) {
    for (int r = 1; r < c->nranks; ++r) {
      int32_t w = 0;
      if (!io_all(c->fd[r], &w, 4, false, c->timeout_ms)) return -1;
      bad += w != 0;
    }
    for (int r = 1; r < c->nranks; ++r)
      if (!io_all(c->fd[r], &bad, 4, true, c->timeout_ms)) return -1;
  } else if (!io_all(c->fd[0], &mine, 4, true, c->timeout_ms) || !io_all(c->fd[0], &bad, 4, false, c->timeout_ms)) {
    return -1;
  }
  return bad;
}

// Non-blocking communicator initialisation with a deadline: a rank whose peers never arrive (or
// whose init fails) aborts its half-built communicator instead of waiting forever.
ncclResult_t init_rank_deadline(gpf_comm* c, const ncclUniqueId& id) {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t nr = ncclCommInitRankConfig(&c->nccl, c->nranks, id, c->rank, &cfg);
  if (nr != ncclSuccess && nr != ncclInProgress) return nr;
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(c->timeout_ms);
  for (;;) {
    ncclResult_t st = ncclInProgress;
    if (ncclCommGetAsyncError(c->nccl, &st) != ncclSuccess) st = ncclInternalError;
    if (st != ncclInProgress) return st;
    if (std::chrono::steady_clock::now() > t_end) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

// Rank 0 -> everyone: n bytes (the ncclUniqueId).
int host_bcast(gpf_comm* c, void* buf, size_t n) {
  if (c->rank == 0) {
    for (int r = 1; r < c->nranks; ++r)
      if (!io_all(c->fd[r], buf, n, true, c->timeout_ms)) return comm_fail(c, "broadcast to rank " + std::to_string(r) + " failed");
  } else if (!io_all(c->fd[0], buf, n, false, c->timeout_ms)) {
    return comm_fail(c, "broadcast from rank 0 failed");
  }
  return GPF_OK;
}

// Star all-reduce over the rendezvous sockets; rank 0 combines in rank order (deterministic).
int host_allreduce(gpf_comm* c, double* buf, int64_t n, int op) {
  const size_t nb = (size_t)n * 8;
  if (c->rank == 0) {
    std::vector<double> in((size_t)n);
    for (int r = 1; r < c->nranks; ++r) {
      if (!io_all(c->fd[r], in.data(), nb, false, c->timeout_ms)) return comm_fail(c, "all-reduce: receive from rank " + std::to_string(r) + " failed");
      for (int64_t i = 0; i < n; ++i) buf[i] = op == GPF_OP_MAX ? std::max(buf[i], in[i]) : buf[i] + in[i];
    }
    for (int r = 1; r < c->nranks; ++r)
      if (!io_all(c->fd[r], buf, nb, true, c->timeout_ms)) return comm_fail(c, "all-reduce: send to rank " + std::to_string(r) + " failed");
  } else {
    if (!io_all(c->fd[0], buf, nb, true, c->timeout_ms) || !io_all(c->fd[0], buf, nb, false, c->timeout_ms))
      return comm_fail(c, "all-reduce: exchange with rank 0 failed");
  }
  return GPF_OK;
}

int rccl_allreduce(gpf_comm* c, double* buf, int64_t n, int op) {
  if (!c->nccl) return comm_fail(c, "all-reduce: the RCCL communicator was aborted after an earlier failure");
  if (hipSetDevice(c->device) != hipSuccess) return comm_fail(c, "all-reduce: hipSetDevice failed");
  if ((size_t)n > c->cap) {
    hipFree(c->d_buf);
    hipHostFree(c->h_buf);
    c->d_buf = nullptr;
    c->h_buf = nullptr;
    c->cap = 0;
    const size_t cap = std::max<size_t>((size_t)n, 1024);
    if (hipMalloc(&c->d_buf, cap * 8) != hipSuccess || hipHostMalloc((void**)&c->h_buf, cap * 8, hipHostMallocDefault) != hipSuccess)
      return comm_fail(c, "all-reduce: staging allocation failed");
    c->cap = cap;
  }
  std::memcpy(c->h_buf, buf, (size_t)n * 8);
  if (hipMemcpyAsync(c->d_buf, c->h_buf, (size_t)n * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return comm_fail(c, "all-reduce: upload failed");
  ncclResult_t nr = ncclAllReduce(c->d_buf, c->d_buf, (size_t)n, ncclFloat64, op == GPF_OP_MAX ? ncclMax : ncclSum,
                                  c->nccl, c->stream);
  // the communicator is non-blocking (init_rank_deadline): an enqueue may report ncclInProgress
  // until RCCL has issued it; the stream synchronisation below then orders the result
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(c->timeout_ms);
  while (nr == ncclInProgress && std::chrono::steady_clock::now() < t_end) {
    if (ncclCommGetAsyncError(c->nccl, &nr) != ncclSuccess) nr = ncclInternalError;
    if (nr == ncclInProgress) std::this_thread::yield();
  }
  if (nr != ncclSuccess) {
    // a collective still in progress at the deadline (or a failed one) stays queued on the
    // stream: abort the communicator so that no later exchange, and not gpf_comm_close's
    // ncclCommDestroy, waits on it or mixes its result in; later calls fail fast
    const std::string why = nr == ncclInProgress ? "timed out" : ncclGetErrorString(nr);
    ncclCommAbort(c->nccl);
    c->nccl = nullptr;
    return comm_fail(c, "ncclAllReduce: " + why + " (communicator aborted)");
  }
  if (hipMemcpyAsync(c->h_buf, c->d_buf, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return comm_fail(c, "all-reduce: download failed");
  std::memcpy(buf, c->h_buf, (size_t)n * 8);
  return GPF_OK;
}

}  // namespace

extern "C" {

int gpf_comm_open(gpf_ctx* ctx, int rank, int nranks, const char* host, int port, int transport, gpf_comm** out) {
  if (!out) return GPF_BAD_ARG;
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && (!host || port <= 0 || port > 65535)) ||
      (transport != GPF_COMM_RCCL && transport != GPF_COMM_HOST) || (transport == GPF_COMM_RCCL && !ctx))
    return GPF_BAD_ARG;
  gpf_comm* c = new gpf_comm();
  c->rank = rank;
  c->nranks = nranks;
  c->transport = transport;
  if (const char* s = getenv("GPF_COMM_TIMEOUT_S")) c->timeout_ms = std::max(1, atoi(s)) * 1000;
  int rc = nranks > 1 ? rendezvous(c, host, port) : GPF_OK;
  if (rc == GPF_OK && transport == GPF_COMM_HOST && nranks > 1) {
    // the host transport runs the same id hand-out as the RCCL one (a stand-in 128-byte id,
    // checked on every rank), so the CPU tests exercise the broadcast the RCCL bootstrap relies on
    unsigned char id[128];
    for (int i = 0; i < 128; ++i) id[i] = (unsigned char)(rank == 0 ? (i * 37 + 11) & 255 : 0);
    rc = host_bcast(c, id, sizeof(id));
    for (int i = 0; rc == GPF_OK && i < 128; ++i)
      if (id[i] != (unsigned char)((i * 37 + 11) & 255)) rc = comm_fail(c, "gpf_comm_open: id broadcast corrupted");
  }
  if (rc == GPF_OK && transport == GPF_COMM_RCCL) {
    // bootstrap in agreed steps (host_agree after each): rank 0's id (with its status word),
    // every rank's stream, then the communicator itself (non-blocking init with a deadline), so a
    // failure on any rank fails every rank at the same step with that rank's message
    c->device = ctx->device;
    struct {
      int32_t status;
      ncclUniqueId id;
    } msg;
    std::memset(&msg, 0, sizeof(msg));
    if (rank == 0) {
      const ncclResult_t nr = ncclGetUniqueId(&msg.id);
      if (nr != ncclSuccess) {
        msg.status = 1;
        comm_fail(c, std::string("ncclGetUniqueId: ") + ncclGetErrorString(nr));
      }
    }
    if (nranks > 1) rc = host_bcast(c, &msg, sizeof(msg));
    if (rc == GPF_OK && msg.status != 0) rc = comm_fail(c, rank == 0 ? c->err : "gpf_comm_open: rank 0 could not create the RCCL id");
    int32_t mine = 0;
    if (rc == GPF_OK &&
        (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)) {
      mine = 1;
      comm_fail(c, "gpf_comm_open: stream creation failed");
    }
    if (rc == GPF_OK) {
      const int nbad = host_agree(c, mine);
      if (nbad != 0) rc = comm_fail(c, mine ? c->err : nbad < 0 ? "gpf_comm_open: rendezvous lost" : "gpf_comm_open: another rank could not create its stream");
    }
    if (rc == GPF_OK) {
      const ncclResult_t nr = init_rank_deadline(c, msg.id);
      mine = nr != ncclSuccess;
      if (mine) {
        comm_fail(c, std::string("ncclCommInitRank: ") + (nr == ncclInProgress ? "timed out" : ncclGetErrorString(nr)));
        if (c->nccl) ncclCommAbort(c->nccl);
        c->nccl = nullptr;
      }
      const int nbad = host_agree(c, mine);
      if (nbad != 0) rc = comm_fail(c, mine ? c->err : nbad < 0 ? "gpf_comm_open: rendezvous lost" : "gpf_comm_open: ncclCommInitRank failed on another rank");
    }
  }
  if (rc != GPF_OK) {
    if (ctx) ctx->err = c->err;
    gpf_comm_close(c);
    return rc;
  }
  *out = c;
  return GPF_OK;
}

void gpf_comm_close(gpf_comm* c) {
  if (!c) return;
  if (c->nccl) ncclCommDestroy(c->nccl);
  if (c->device >= 0) hipSetDevice(c->device);
  if (c->stream) hipStreamDestroy(c->stream);
  hipFree(c->d_buf);
  hipHostFree(c->h_buf);
  for (int f : c->fd)
    if (f >= 0) close(f);
  delete c;
}

int gpf_comm_rank(const gpf_comm* c) { return c ? c->rank : -1; }
int gpf_comm_stats(const gpf_comm* c, double* exchange_ms, long long* exchanges) {
  if (!c) return GPF_BAD_ARG;
  if (exchange_ms) *exchange_ms = c->xch_ms;
  if (exchanges) *exchanges = c->xch_n;
  return GPF_OK;
}
int gpf_comm_size(const gpf_comm* c) { return c ? c->nranks : -1; }
const char* gpf_comm_last_error(const gpf_comm* c) { return c ? c->err.c_str() : "null communicator"; }

int gpf_comm_allreduce(gpf_comm* c, double* buf, int64_t n, int op) {
  if (!c || n < 0 || (n > 0 && !buf) || (op != GPF_OP_SUM && op != GPF_OP_MAX)) return GPF_BAD_ARG;
  if (n == 0) return GPF_OK;
  if (c->transport == GPF_COMM_RCCL) return rccl_allreduce(c, buf, n, op);
  return c->nranks > 1 ? host_allreduce(c, buf, n, op) : GPF_OK;
}

int gpf_comm_exchange_scores(gpf_comm* c, int P, const double* local, int local_rc, int local_bad, double* loss,
                             int* bad_idx) {
  if (!c || P < 0 || !loss) return GPF_BAD_ARG;
  if (bad_idx) *bad_idx = -1;
  const int G = c->nranks, r = c->rank;
  const int lo = (int)((long long)r * P / G), hi = (int)((long long)(r + 1) * P / G);
  std::vector<double> buf((size_t)P + G, 0.0);
  if (local_rc == GPF_OK) {
    if (hi > lo && !local) return GPF_BAD_ARG;
    for (int i = lo; i < hi; ++i) buf[i] = local[i - lo];
  } else {
    buf[(size_t)P + r] = local_rc == GPF_NOT_PD ? 1.0 + (double)(lo + std::max(local_bad, 0)) : -(double)local_rc;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const int arc = gpf_comm_allreduce(c, buf.data(), (int64_t)buf.size(), GPF_OP_SUM);
  c->xch_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ++c->xch_n;
  if (arc) return arc;
  int bad = -1, failed = -1, code = GPF_OK;
  for (int q = 0; q < G; ++q) {
    const double s = buf[(size_t)P + q];
    if (s > 0.0 && bad < 0) bad = (int)(s - 1.0);  // ranks own ascending rows: the first is the smallest
    if (s < 0.0 && failed < 0) {
      failed = q;
      code = (int)(-s);
    }
  }
  if (failed >= 0) {
    c->err = "rank " + std::to_string(failed) + " failed to score its particles (code " + std::to_string(code) + ")";
    return code == GPF_BAD_ARG ? GPF_BAD_ARG : GPF_HIP_ERROR;
  }
  if (bad >= 0) {
    if (bad_idx) *bad_idx = bad;
    c->err = "Matrix is not positive definite";
    return GPF_NOT_PD;
  }
  std::memcpy(loss, buf.data(), (size_t)P * 8);
  return GPF_OK;
}

int gpf_eval_batch_sharded(gpf_ctx* ctx, gpf_comm* c, const double* ls, int P, double* loss, int* bad_idx) {
  if (!ctx || !c || P < 0 || (P > 0 && (!ls || !loss))) return GPF_BAD_ARG;
  if (bad_idx) *bad_idx = -1;
  const int G = c->nranks, r = c->rank;
  const int lo = (int)((long long)r * P / G), hi = (int)((long long)(r + 1) * P / G);
  std::vector<double> part((size_t)std::max(hi - lo, 0));
  int bad = -1, rc = GPF_OK;
  if (hi > lo) rc = gpf_eval_batch(ctx, ls + (size_t)lo * ctx->d, hi - lo, part.data(), nullptr, nullptr, &bad);
  const std::string local_err = rc != GPF_OK ? ctx->err : std::string();
  const int xr = gpf_comm_exchange_scores(c, P, part.data(), rc, bad, loss, bad_idx);
  if (xr != GPF_OK) ctx->err = local_err.empty() ? c->err : local_err;
  return xr;
}

}  // extern "C"
