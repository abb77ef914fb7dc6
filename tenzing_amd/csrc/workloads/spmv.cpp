#include "workloads.hpp"
#include "core/solve.hpp"

#include "core/util.hpp"
#include "hip/hip_runtime.hpp"
#include "hip/rccl_comm.hpp"
#include "hip/rocsparse_spmv.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>

namespace tz {

Json SpmvArgs::json() const {
  Json j;
  j["m"] = m;
  j["bw"] = bw;
  j["nnz"] = nnz;
  j["nnz_actual"] = nnz_actual;
  j["seed"] = int64_t(seed);
  j["rank"] = rank;
  j["size"] = size;
  j["compound"] = compound;
  j["kernel_choice"] = kernel_choice;
  j["form"] = form;
  j["library"] = library;
  j["transport"] = transport;
  j["matrix"] = matrix;
  j["distribute"] = distribute;
  return j;
}

CsrHost random_band_matrix(int64_t n, int64_t bw, int64_t nnz, uint64_t seed) {
  // The reference's generator (include/tenzing/spmv/csr_mat.hpp:334-370): a row uniformly at
  // random, a column uniformly in [r - bw, r + bw] (draws outside the matrix are dropped, not
  // clamped, so the first and last columns are not over-weighted), duplicates removed, and
  // refilled until exactly nnz distinct entries exist. Values here are uniform in [-1, 1)
  // (the reference stores 1.0) so that a wrong column shows in the numerical check.
  TZ_CHECK(n > 0 && bw >= 0 && nnz >= 0, "bad band matrix parameters");
  int64_t capacity = 0; // entries inside the band
  for (int64_t r = 0; r < n && capacity < nnz; ++r)
    capacity += std::min(n - 1, r + bw) - std::max<int64_t>(0, r - bw) + 1;
  TZ_CHECK(nnz <= capacity, "nnz " << nnz << " exceeds the " << capacity << " entries of an " << n
                                    << " x " << n << " band of half-width " << bw);
  std::mt19937_64 rng(seed);
  const uint64_t width = uint64_t(2 * bw + 1);
  std::vector<int64_t> keys;
  keys.reserve(size_t(nnz));
  while (int64_t(keys.size()) < nnz) {
    const int64_t need = nnz - int64_t(keys.size());
    for (int64_t k = 0; k < need; ++k) {
      const int64_t r = int64_t(rng() % uint64_t(n));
      const int64_t c = r - bw + int64_t(rng() % width);
      if (c < 0 || c >= n) continue;
      keys.push_back(r * n + c);
    }
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  }
  CsrHost A;
  A.rows = A.cols = n;
  A.rowPtr.assign(size_t(n + 1), 0);
  A.colInd.reserve(keys.size());
  A.val.reserve(keys.size());
  std::mt19937_64 vrng(seed ^ 0x9E3779B97F4A7C15ull);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  for (int64_t key : keys) {
    const int64_t r = key / n, c = key % n;
    A.rowPtr[size_t(r + 1)]++;
    A.colInd.push_back(int32_t(c));
    A.val.push_back(u(vrng));
  }
  for (int64_t r = 0; r < n; ++r) A.rowPtr[size_t(r + 1)] += A.rowPtr[size_t(r)];
  return A;
}

CsrHost read_matrix_market(const std::string &path) {
  std::ifstream f(path);
  TZ_CHECK(f, "cannot open " << path);
  std::string line;
  TZ_CHECK(std::getline(f, line), path << ": empty file");
  std::istringstream hs(line);
  std::string banner, object, format, field, symmetry;
  hs >> banner >> object >> format >> field >> symmetry;
  auto lower = [](std::string v) {
    std::transform(v.begin(), v.end(), v.begin(), [](unsigned char c) { return char(std::tolower(c)); });
    return v;
  };
  object = lower(object), format = lower(format), field = lower(field), symmetry = lower(symmetry);
  TZ_CHECK(banner == "%%MatrixMarket" && object == "matrix", path << ": not a Matrix Market matrix");
  TZ_CHECK(format == "coordinate", path << ": only coordinate (sparse) format is supported");
  TZ_CHECK(field == "real" || field == "integer" || field == "pattern" || field == "double",
           path << ": unsupported field " << field);
  TZ_CHECK(symmetry == "general" || symmetry == "symmetric" || symmetry == "skew-symmetric",
           path << ": unsupported symmetry " << symmetry);
  while (std::getline(f, line))
    if (!line.empty() && line[0] != '%') break;
  int64_t rows = 0, cols = 0, entries = 0;
  {
    std::istringstream ss(line);
    TZ_CHECK(ss >> rows >> cols >> entries, path << ": bad size line");
  }
  TZ_CHECK(rows > 0 && cols > 0 && entries >= 0 && rows < (int64_t(1) << 31) && cols < (int64_t(1) << 31),
           path << ": bad dimensions");
  // CsrHost::rowPtr is int32: the stored entries (off-diagonal ones twice for symmetric files)
  // must fit, or the row pointers would overflow silently
  const int64_t most = symmetry == "general" ? entries : 2 * entries;
  TZ_CHECK(most < (int64_t(1) << 31) - 1,
           path << ": " << most << " stored entries (after symmetric expansion) exceed the int32 CSR "
                << "row pointers");
  std::vector<std::pair<int64_t, float>> e; // (row * cols + col, value)
  e.reserve(size_t(entries) * (symmetry == "general" ? 1 : 2));
  for (int64_t k = 0; k < entries; ++k) {
    do {
      TZ_CHECK(std::getline(f, line), path << ": " << k << " of " << entries << " entries");
    } while (line.empty() || line[0] == '%');
    std::istringstream ss(line);
    int64_t r = 0, c = 0;
    double v = 1.0;
    TZ_CHECK(ss >> r >> c, path << ": bad entry line " << line);
    if (field != "pattern") TZ_CHECK(ss >> v, path << ": entry without a value: " << line);
    TZ_CHECK(r >= 1 && r <= rows && c >= 1 && c <= cols, path << ": entry out of range: " << line);
    --r, --c;
    e.emplace_back(r * cols + c, float(v));
    if (symmetry != "general" && r != c) e.emplace_back(c * cols + r, float(symmetry == "symmetric" ? v : -v));
  }
  std::sort(e.begin(), e.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
  CsrHost A;
  A.rows = rows;
  A.cols = cols;
  A.rowPtr.assign(size_t(rows + 1), 0);
  for (size_t k = 0; k < e.size(); ++k) {
    if (k > 0 && e[k].first == e[k - 1].first) {
      A.val.back() += e[k].second; // duplicates add up
      continue;
    }
    A.rowPtr[size_t(e[k].first / cols + 1)]++;
    A.colInd.push_back(int32_t(e[k].first % cols));
    A.val.push_back(e[k].second);
  }
  for (int64_t r = 0; r < rows; ++r) A.rowPtr[size_t(r + 1)] += A.rowPtr[size_t(r)];
  return A;
}

void write_matrix_market(const CsrHost &A, const std::string &path) {
  std::ofstream f(path);
  TZ_CHECK(f, "cannot write " << path);
  f << "%%MatrixMarket matrix coordinate real general\n";
  f << A.rows << " " << A.cols << " " << A.nnz() << "\n";
  f.precision(9);
  for (int64_t r = 0; r < A.rows; ++r)
    for (int32_t j = A.rowPtr[size_t(r)]; j < A.rowPtr[size_t(r + 1)]; ++j)
      f << r + 1 << " " << A.colInd[size_t(j)] + 1 << " " << A.val[size_t(j)] << "\n";
  TZ_CHECK(f.good(), "write to " << path << " failed");
}

std::pair<int64_t, int64_t> row_partition(int64_t n, int rank, int size) {
  const int64_t base = n / size, rem = n % size;
  const int64_t r0 = rank * base + std::min<int64_t>(rank, rem);
  return {r0, r0 + base + (rank < rem ? 1 : 0)};
}

static int owner_of(int64_t col, int64_t n, int size) {
  // inverse of row_partition
  const int64_t base = n / size, rem = n % size;
  const int64_t cut = rem * (base + 1);
  if (col < cut) return int(col / (base + 1));
  return int(rem + (col - cut) / std::max<int64_t>(base, 1));
}

static float x_value(int64_t g) { return float(int64_t((uint64_t(g) * 2654435761ull) % 2000ull) - 1000) / 1000.f; }

namespace {

class SpmvLocal : public GpuOp {
public:
  SpmvLocal(std::shared_ptr<const DistSpmv> s, std::string name, int lanes, bool intoY)
      : s_(std::move(s)), name_(std::move(name)), lanes_(lanes), intoY_(intoY) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvLocal"; }
  double bytes() const override { return 12.0 * double(s_->local_nnz()) + 8.0 * double(s_->local_rows()); }
  double cost_us() const override { return 4.0 + bytes() / 3.0e6; }
  void launch(void *st, Executor &) const override { s_->spmv_local(lanes_, st, intoY_); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
  int lanes_;
  bool intoY_;
};

class SpmvRemote : public GpuOp {
public:
  SpmvRemote(std::shared_ptr<const DistSpmv> s, std::string name, bool accumulate)
      : s_(std::move(s)), name_(std::move(name)), acc_(accumulate) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvRemote"; }
  double bytes() const override {
    return s_->remote_nnz() ? 12.0 * double(s_->remote_nnz()) + 8.0 * double(s_->local_rows()) : 0.0;
  }
  double cost_us() const override { return s_->remote_nnz() ? 4.0 + bytes() / 3.0e6 : 0.5; }
  void launch(void *st, Executor &) const override { s_->spmv_remote(st, acc_); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
  bool acc_;
};

class SpmvScatter : public GpuOp {
public:
  SpmvScatter(std::shared_ptr<const DistSpmv> s, std::string name) : s_(std::move(s)), name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvScatter"; }
  double cost_us() const override { return s_->send_elems() ? 3.0 + 12.0 * double(s_->send_elems()) / 2.0e6 : 0.5; }
  void launch(void *st, Executor &) const override { s_->scatter(st); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
};

class SpmvExchange : public GpuOp {
public:
  SpmvExchange(std::shared_ptr<const DistSpmv> s, std::string name) : s_(std::move(s)), name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvExchange"; }
  double cost_us() const override { return s_->num_peers() ? 10.0 + 4.0 * double(s_->send_elems()) / 5.0e4 : 0.5; }
  std::string order_domain() const override { return s_->uses_rccl() ? "rccl" : ""; }
  bool capturable() const override { return !s_->uses_rccl() || s_->rccl_graph_ok(); }
  void launch(void *st, Executor &) const override { s_->exchange(st); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
};

/// ipc transport: gather my x entries straight into the peers' remote-x buffers (+ signals)
class SpmvPut : public GpuOp {
public:
  SpmvPut(std::shared_ptr<const DistSpmv> s, std::string name) : s_(std::move(s)), name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvPut"; }
  double cost_us() const override { return s_->num_peers() ? 6.0 + 4.0 * double(s_->send_elems()) / 5.0e4 : 0.5; }
  void launch(void *st, Executor &) const override { s_->put(st); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
};

/// ipc transport: device-side wait for the peers' puts into my remote-x buffer
class SpmvWait : public GpuOp {
public:
  SpmvWait(std::shared_ptr<const DistSpmv> s, std::string name) : s_(std::move(s)), name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvWait"; }
  double cost_us() const override { return 3.0; }
  void launch(void *st, Executor &) const override { s_->wait_puts(st); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
};

/// ipc transport: remote product, then the senders' credits go back
class SpmvRemoteRelease : public GpuOp {
public:
  SpmvRemoteRelease(std::shared_ptr<const DistSpmv> s, std::string name, bool accumulate)
      : s_(std::move(s)), name_(std::move(name)), acc_(accumulate) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "SpmvRemote"; }
  double cost_us() const override { return s_->remote_nnz() ? 6.0 + 12.0 * double(s_->remote_nnz()) / 3.0e6 : 2.5; }
  void launch(void *st, Executor &) const override {
    s_->spmv_remote(st, acc_);
    s_->release(st);
  }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
  bool acc_;
};

class SpmvAdd : public GpuOp {
public:
  SpmvAdd(std::shared_ptr<const DistSpmv> s, std::string name) : s_(std::move(s)), name_(std::move(name)) {}
  std::string name() const override { return name_; }
  std::string kind() const override { return "VectorAdd"; }
  double cost_us() const override { return 3.0 + 12.0 * double(s_->local_rows()) / 4.0e6; }
  void launch(void *st, Executor &) const override { s_->add(st); }

private:
  std::shared_ptr<const DistSpmv> s_;
  std::string name_;
};

} // namespace

namespace {
// (de)serialization of plain arrays for the setup messages
template <typename T> void put_vec(std::string &s, const std::vector<T> &v) {
  const uint64_t n = v.size();
  s.append(reinterpret_cast<const char *>(&n), sizeof(n));
  if (n) s.append(reinterpret_cast<const char *>(v.data()), n * sizeof(T));
}
template <typename T> std::vector<T> get_vec(const std::string &s, size_t &at) {
  uint64_t n = 0;
  TZ_CHECK(at + sizeof(n) <= s.size(), "spmv setup message truncated");
  std::memcpy(&n, s.data() + at, sizeof(n));
  at += sizeof(n);
  TZ_CHECK(at + n * sizeof(T) <= s.size(), "spmv setup message truncated");
  std::vector<T> v(n);
  if (n) std::memcpy(v.data(), s.data() + at, n * sizeof(T));
  at += n * sizeof(T);
  return v;
}
// rows [r0, r1) of A as a CSR of their own (row pointers from 0, global columns)
CsrHost row_block(const CsrHost &A, int64_t r0, int64_t r1) {
  CsrHost B;
  B.rows = r1 - r0;
  B.cols = A.cols;
  B.rowPtr.assign(size_t(B.rows + 1), 0);
  const int32_t base = A.rowPtr[size_t(r0)];
  for (int64_t r = r0; r <= r1; ++r) B.rowPtr[size_t(r - r0)] = A.rowPtr[size_t(r)] - base;
  B.colInd.assign(A.colInd.begin() + base, A.colInd.begin() + A.rowPtr[size_t(r1)]);
  B.val.assign(A.val.begin() + base, A.val.begin() + A.rowPtr[size_t(r1)]);
  return B;
}
} // namespace

CsrHost DistSpmv::build_matrix() {
  CsrHost A;
  if (!a_.matrix.empty()) {
    A = read_matrix_market(a_.matrix);
    TZ_CHECK(A.rows == A.cols, a_.matrix << ": the SpMV workload needs a square matrix (x is "
                                          "partitioned like the rows), got " << A.rows << " x " << A.cols);
    a_.m = A.rows;
    a_.nnz = A.nnz();
    a_.bw = 0;
  } else {
    if (a_.bw <= 0) a_.bw = std::max<int64_t>(1, a_.m / a_.size);
    if (a_.nnz <= 0) a_.nnz = 10 * a_.m;
    A = random_band_matrix(a_.m, a_.bw, a_.nnz, a_.seed);
  }
  a_.nnz_actual = A.nnz();
  return A;
}

DistSpmv::DistSpmv(SpmvArgs a, Ctrl *ctrl) : a_(std::move(a)) {
  TZ_CHECK(a_.size >= 1 && a_.rank >= 0 && a_.rank < a_.size, "bad rank/size");
  TZ_CHECK(a_.distribute == "local" || a_.distribute == "root" || a_.distribute == "auto",
           "SpMV distribute must be local, root or auto (got " << a_.distribute << ")");
  if (a_.distribute == "auto") a_.distribute = ctrl && a_.size > 1 ? "root" : "local";
  const bool root = a_.distribute == "root" && a_.size > 1;
  TZ_CHECK(!root || (ctrl && ctrl->size() == a_.size && ctrl->rank() == a_.rank),
           "SpMV root distribution needs the control plane of its " << a_.size << " ranks");
  CsrHost mine; // my rows, global columns
  // needFrom[q]: the global columns of mine that rank q's rows use (what I send q, in q's order)
  std::vector<std::vector<int64_t>> needFrom(size_t(a_.size));
  if (!root) {
    // every rank derives the same matrix and every plan itself (no setup communication)
    const CsrHost A = build_matrix();
    TZ_CHECK(a_.m >= a_.size, "fewer matrix rows (" << a_.m << ") than ranks (" << a_.size << ")");
    std::tie(r0_, r1_) = row_partition(a_.m, a_.rank, a_.size);
    mine = row_block(A, r0_, r1_);
    for (int q = 0; q < a_.size; ++q) {
      if (q == a_.rank) continue;
      auto [q0, q1] = row_partition(a_.m, q, a_.size);
      std::vector<int64_t> &need = needFrom[size_t(q)];
      for (int64_t r = q0; r < q1; ++r)
        for (int32_t j = A.rowPtr[r]; j < A.rowPtr[r + 1]; ++j)
          if (A.colInd[j] >= r0_ && A.colInd[j] < r1_) need.push_back(A.colInd[j]);
      std::sort(need.begin(), need.end());
      need.erase(std::unique(need.begin(), need.end()), need.end());
    }
  } else {
    // the reference's setup (include/tenzing/spmv/row_part_spmv.cuh:24-90, :322-403): rank 0
    // builds (or reads) the matrix and sends every rank its row block; then every rank tells
    // each owner which of its columns it needs, and each owner builds its send plan from that
    // A failure on rank 0 (a missing or malformed matrix file, nnz above the band's capacity,
    // fewer rows than ranks) travels in the row-block header (hdr[4] = 1, then the message), so
    // every rank throws the same error right after this exchange instead of waiting in it
    std::vector<std::string> out(size_t(a_.size));
    if (a_.rank == 0) {
      std::string err;
      try {
        const CsrHost A = build_matrix();
        TZ_CHECK(a_.m >= a_.size, "fewer matrix rows (" << a_.m << ") than ranks (" << a_.size << ")");
        for (int q = 0; q < a_.size; ++q) {
          auto [q0, q1] = row_partition(a_.m, q, a_.size);
          const CsrHost B = row_block(A, q0, q1);
          std::string &m = out[size_t(q)];
          const int64_t hdr[5] = {a_.m, a_.nnz, a_.bw, a_.nnz_actual, 0};
          m.append(reinterpret_cast<const char *>(hdr), sizeof(hdr));
          put_vec(m, B.rowPtr);
          put_vec(m, B.colInd);
          put_vec(m, B.val);
        }
      } catch (const std::exception &e) {
        err = e.what();
      }
      if (!err.empty())
        for (std::string &m : out) {
          const int64_t hdr[5] = {0, 0, 0, 0, 1};
          m.assign(reinterpret_cast<const char *>(hdr), sizeof(hdr));
          m += err;
        }
    }
    const std::vector<std::string> in = ctrl->alltoallv(out);
    const std::string &msg = in[0];
    int64_t hdr[5];
    TZ_CHECK(msg.size() >= sizeof(hdr), "spmv setup: no row block from rank 0");
    std::memcpy(hdr, msg.data(), sizeof(hdr));
    TZ_CHECK(hdr[4] == 0, "spmv setup on rank 0 failed: " << msg.substr(sizeof(hdr)));
    a_.m = hdr[0];
    a_.nnz = hdr[1];
    a_.bw = hdr[2];
    a_.nnz_actual = hdr[3];
    size_t at = sizeof(hdr);
    std::tie(r0_, r1_) = row_partition(a_.m, a_.rank, a_.size);
    mine.rows = r1_ - r0_;
    mine.cols = a_.m;
    mine.rowPtr = get_vec<int32_t>(msg, at);
    mine.colInd = get_vec<int32_t>(msg, at);
    mine.val = get_vec<float>(msg, at);
    TZ_CHECK(int64_t(mine.rowPtr.size()) == mine.rows + 1, "spmv setup: row block of the wrong size");
    // column requests: to each owner, the sorted columns of its I need
    std::vector<std::vector<int64_t>> want(size_t(a_.size));
    for (int32_t c : mine.colInd)
      if (c < r0_ || c >= r1_) want[size_t(owner_of(c, a_.m, a_.size))].push_back(c);
    std::vector<std::string> req(size_t(a_.size));
    for (int q = 0; q < a_.size; ++q) {
      std::vector<int64_t> &w = want[size_t(q)];
      std::sort(w.begin(), w.end());
      w.erase(std::unique(w.begin(), w.end()), w.end());
      put_vec(req[size_t(q)], w);
    }
    const std::vector<std::string> got = ctrl->alltoallv(req);
    for (int q = 0; q < a_.size; ++q) {
      if (q == a_.rank) continue;
      size_t k = 0;
      needFrom[size_t(q)] = get_vec<int64_t>(got[size_t(q)], k);
      for (int64_t c : needFrom[size_t(q)])
        TZ_CHECK(c >= r0_ && c < r1_, "spmv setup: rank " << q << " asked for column " << c << ", not mine");
    }
  }
  const int64_t n = a_.m;

  // split my rows into local (own x) and remote (others' x) blocks
  std::vector<int64_t> rc;
  for (int32_t c : mine.colInd)
    if (c < r0_ || c >= r1_) rc.push_back(c);
  std::sort(rc.begin(), rc.end());
  rc.erase(std::unique(rc.begin(), rc.end()), rc.end());
  remoteCols_ = rc;

  const int64_t nl = r1_ - r0_;
  local_.rows = remote_.rows = nl;
  local_.cols = nl;
  remote_.cols = int64_t(rc.size());
  local_.rowPtr.assign(size_t(nl + 1), 0);
  remote_.rowPtr.assign(size_t(nl + 1), 0);
  yRef_.assign(size_t(nl), 0.0);
  for (int64_t i = 0; i < nl; ++i) {
    double acc = 0;
    for (int32_t j = mine.rowPtr[size_t(i)]; j < mine.rowPtr[size_t(i + 1)]; ++j) {
      const int64_t c = mine.colInd[size_t(j)];
      acc += double(mine.val[size_t(j)]) * double(x_value(c));
      if (c >= r0_ && c < r1_) {
        local_.colInd.push_back(int32_t(c - r0_));
        local_.val.push_back(mine.val[size_t(j)]);
      } else {
        const int64_t p = std::lower_bound(rc.begin(), rc.end(), c) - rc.begin();
        remote_.colInd.push_back(int32_t(p));
        remote_.val.push_back(mine.val[size_t(j)]);
      }
    }
    yRef_[size_t(i)] = acc;
    local_.rowPtr[size_t(i + 1)] = int32_t(local_.colInd.size());
    remote_.rowPtr[size_t(i + 1)] = int32_t(remote_.colInd.size());
  }

  // receive plan: remote cols are sorted, hence grouped by owner
  recvCount_.assign(size_t(a_.size), 0);
  recvOff_.assign(size_t(a_.size), 0);
  for (int64_t c : rc) recvCount_[size_t(owner_of(c, n, a_.size))]++;
  for (int q = 1; q < a_.size; ++q) recvOff_[q] = recvOff_[q - 1] + recvCount_[q - 1];

  // send plan: what every other rank q needs from my columns, in q's (sorted) order
  sendCount_.assign(size_t(a_.size), 0);
  sendOff_.assign(size_t(a_.size), 0);
  for (int q = 0; q < a_.size; ++q) {
    sendOff_[q] = int32_t(sendIdx_.size());
    for (int64_t c : needFrom[size_t(q)]) sendIdx_.push_back(int32_t(c - r0_));
    sendCount_[q] = int32_t(needFrom[size_t(q)].size());
  }
  xLocal_.resize(size_t(nl));
  for (int64_t i = 0; i < nl; ++i) xLocal_[size_t(i)] = x_value(r0_ + i);
  TZ_CHECK(a_.transport == "auto" || a_.transport == "rccl" || a_.transport == "ipc",
           "SpMV transport must be auto, rccl or ipc (got " << a_.transport << ")");
  useRccl_ = a_.size > 1 && a_.transport != "ipc";
  useIpc_ = a_.size > 1 && a_.transport != "rccl";
  const double avg = nl ? double(local_.nnz() + remote_.nnz()) / double(nl) : 1;
  lanes_ = avg > 24 ? 16 : (avg > 6 ? 8 : 4);
}

DistSpmv::~DistSpmv() {
  for (void *p : opened_) (void)hipIpcCloseMemHandle(p);
  if (flags_) (void)hipFree(flags_);
}

std::string DistSpmv::transport() const {
  if (a_.size == 1) return "none";
  std::string t;
  if (useRccl_) t = "rccl";
  if (useIpc_ && (ipcReady_ || !ready())) t += t.empty() ? "ipc" : "+ipc";
  return t.empty() ? "none" : t;
}

int DistSpmv::num_peers() const {
  int n = 0;
  for (int q = 0; q < a_.size; ++q) n += (recvCount_[q] > 0 || sendCount_[q] > 0);
  return n;
}

void DistSpmv::setup(Ctrl *ctrl) {
  if (ready()) return;
  if (a_.device >= 0) TZ_HIP(hipSetDevice(a_.device));
  auto up = [](DeviceBuffer &d, const void *p, size_t bytes) {
    d = DeviceBuffer(std::max<size_t>(bytes, 16));
    d.upload(p, bytes);
  };
  up(dLocalRow_, local_.rowPtr.data(), local_.rowPtr.size() * 4);
  up(dLocalCol_, local_.colInd.data(), local_.colInd.size() * 4);
  up(dLocalVal_, local_.val.data(), local_.val.size() * 4);
  up(dRemoteRow_, remote_.rowPtr.data(), remote_.rowPtr.size() * 4);
  up(dRemoteCol_, remote_.colInd.data(), remote_.colInd.size() * 4);
  up(dRemoteVal_, remote_.val.data(), remote_.val.size() * 4);
  up(dX_, xLocal_.data(), xLocal_.size() * 4);
  up(dSendIdx_, sendIdx_.data(), sendIdx_.size() * 4);
  const size_t nl = size_t(local_rows());
  dSend_ = DeviceBuffer(std::max<size_t>(sendIdx_.size() * 4, 16));
  // (at least 64 KB: an IPC-exported buffer of its own rather than a sub-allocation)
  dXr_ = DeviceBuffer(std::max<size_t>(remoteCols_.size() * 4, 65536), /*peerWritten=*/useIpc_);
  dYl_ = DeviceBuffer(std::max<size_t>(nl * 4, 16));
  dYr_ = DeviceBuffer(std::max<size_t>(nl * 4, 16));
  dY_ = DeviceBuffer(std::max<size_t>(nl * 4, 16));
  TZ_HIP(hipMemset(dYr_.get(), 0, dYr_.bytes()));
  if (a_.size > 1) {
    TZ_CHECK(ctrl && ctrl->size() == a_.size, "SpMV needs a control plane of size " << a_.size);
    // IPC first (collective agreement, preflight), then RCCL with the same collective fallback
    // as the halo: several ranks on one GPU (loopback) have no RCCL
    if (useIpc_) {
      const std::string why = setup_ipc(ctrl);
      double failed = why.empty() ? 0.0 : 1.0;
      ctrl->allreduce_max(&failed, 1);
      ipcReady_ = failed == 0.0;
      if (!ipcReady_) {
        TZ_LOG(Warn, "SpMV ipc transport unavailable" << (why.empty() ? " on another rank" : ": " + why));
        TZ_CHECK(a_.transport != "ipc", "SpMV ipc transport requested but unavailable: " << why);
      }
    }
    if (useIpc_ && ipcReady_) {
      TZ_HIP(hipDeviceSynchronize());
      ctrl->barrier();
      ipc_preflight(ctrl);
    }
    if (useRccl_) {
      int dev = 0;
      TZ_HIP(hipGetDevice(&dev));
      std::string why;
      try {
        comm_ = std::make_shared<RcclComm>(*ctrl, dev);
      } catch (const std::exception &e) {
        why = e.what();
        comm_.reset();
      }
      double failed = why.empty() ? 0.0 : 1.0;
      ctrl->allreduce_max(&failed, 1);
      if (failed == 0.0) {
        // one verified exchange before the search may use it, bounded like the halo's
        why = rccl_preflight_local();
        failed = why.empty() ? 0.0 : 1.0;
        ctrl->allreduce_max(&failed, 1);
        if (failed != 0.0) why = "preflight: " + (why.empty() ? std::string("failed on another rank") : why);
        else rccl_graph_preflight(*ctrl);
      }
      if (failed != 0.0) {
        if (comm_ && !comm_->aborted()) comm_->abort();
        comm_.reset();
        TZ_LOG(Warn, "SpMV RCCL transport unavailable" << (why.empty() ? " on another rank" : ": " + why));
        TZ_CHECK(a_.transport == "auto" && useIpc_ && ipcReady_,
                 "SpMV RCCL transport unavailable and no IPC fallback: " << why);
        useRccl_ = false;
      }
    }
  }
  if (a_.kernel_choice && !a_.library.empty() && local_.nnz() > 0) {
    auto mk = [&](DeviceBuffer &y) {
      return std::make_shared<RocsparseCsr>(nl, nl, local_.nnz(), dLocalRow_.as<int32_t>(),
                                            dLocalCol_.as<int32_t>(), dLocalVal_.as<float>(),
                                            dX_.as<float>(), y.as<float>(), a_.library.c_str());
    };
    rsYl_ = mk(dYl_);
    rsY_ = mk(dY_);
  }
  TZ_HIP(hipDeviceSynchronize());
}

void DistSpmv::reset_y(void *stream) {
  // synchronous: schedules run on non-blocking streams that do not order after `stream`
  TZ_HIP(hipMemsetAsync(dY_.get(), 0, dY_.bytes(), static_cast<hipStream_t>(stream)));
  TZ_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

double DistSpmv::check(void *stream) {
  TZ_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  std::vector<float> y(static_cast<size_t>(local_rows()));
  dY_.download(y.data(), y.size() * 4);
  double err = 0;
  for (size_t i = 0; i < y.size(); ++i)
    err = std::max(err, std::abs(double(y[i]) - yRef_[i]) / std::max(1.0, std::abs(yRef_[i])));
  return err;
}

void DistSpmv::scatter(void *stream) const {
  if (sendIdx_.empty()) return; // nothing any peer needs (e.g. one rank)
  kern::gather_f32(int(sendIdx_.size()), dX_.as<float>(), dSendIdx_.as<int32_t>(), dSend_.as<float>(), stream);
}

void DistSpmv::exchange(void *stream) const {
  if (!comm_) return;
  std::vector<RcclComm::Xfer> xs;
  for (int q = 0; q < a_.size; ++q) {
    if (q == a_.rank || (sendCount_[q] == 0 && recvCount_[q] == 0)) continue;
    RcclComm::Xfer x;
    x.send = dSend_.as<float>() + sendOff_[q];
    x.sendCount = size_t(sendCount_[q]);
    x.sendPeer = q;
    x.recv = dXr_.as<float>() + recvOff_[q];
    x.recvCount = size_t(recvCount_[q]);
    x.recvPeer = q;
    xs.push_back(x);
  }
  comm_->exchange(xs, 0, stream);
}

void DistSpmv::spmv_local(int lanes, void *stream, bool intoY) const {
  if (lanes == kLibrary) {
    const auto &rs = intoY ? rsY_ : rsYl_;
    if (rs) {
      rs->run(stream);
      return;
    }
    // no library state only for an empty local block: any kernel writes the zeros
    TZ_CHECK(local_.nnz() == 0, "rocSPARSE SpMV variant not set up");
    lanes = 0;
  }
  kern::csr_spmv(int(local_rows()), dLocalRow_.as<int32_t>(), dLocalCol_.as<int32_t>(),
                 dLocalVal_.as<float>(), dX_.as<float>(), (intoY ? dY_ : dYl_).as<float>(),
                 lanes > 0 ? lanes : lanes_, false, stream);
}

kern::SpmvJob DistSpmv::local_job(int lanes, bool intoY) const {
  TZ_CHECK(ready(), "spmv not set up");
  kern::SpmvJob j;
  j.nRows = int(local_rows());
  j.rowPtr = dLocalRow_.as<int32_t>();
  j.colInd = dLocalCol_.as<int32_t>();
  j.val = dLocalVal_.as<float>();
  j.x = dX_.as<float>();
  j.y = (intoY ? dY_ : dYl_).as<float>();
  j.lanes = lanes;
  j.accumulate = false;
  return j;
}

void DistSpmv::spmv_remote(void *stream, bool accumulate) const {
  // an empty remote block leaves y_r at the zeros set up once (split form) and adds nothing
  // (accumulate form)
  if (remote_.nnz() == 0) return;
  kern::csr_spmv(int(local_rows()), dRemoteRow_.as<int32_t>(), dRemoteCol_.as<int32_t>(),
                 dRemoteVal_.as<float>(), dXr_.as<float>(), (accumulate ? dY_ : dYr_).as<float>(),
                 lanes_, accumulate, stream);
}

// ------------------------------------------------------------------ ipc transport

std::string DistSpmv::setup_ipc(Ctrl *ctrl) {
  // Collective like the halo's: every rank makes the same control-plane calls whatever fails
  // locally. Exported per rank: [flags][remote-x buffer][my recvOff_ per rank (i32)].
  const size_t H = sizeof(hipIpcMemHandle_t);
  const size_t P = size_t(a_.size);
  std::string mine, err;
  if (const char *v = std::getenv("TZ_IPC_TIMEOUT")) ipcTimeoutS_ = std::atof(v);
  try {
    TZ_HIP(hipExtMallocWithFlags(&flags_, std::max<size_t>(2 * P * 8, 64), hipDeviceMallocUncached));
    TZ_HIP(hipMemset(flags_, 0, 2 * P * 8));
    expected_ = DeviceBuffer(P * 8);
    sent_ = DeviceBuffer(P * 8);
    done_ = DeviceBuffer(size_t(kern::kMaxPutPeers) * sizeof(unsigned int));
    err_ = DeviceBuffer(sizeof(int));
    TZ_HIP(hipMemset(expected_.get(), 0, P * 8));
    TZ_HIP(hipMemset(sent_.get(), 0, P * 8));
    TZ_HIP(hipMemset(done_.get(), 0, done_.bytes()));
    TZ_HIP(hipMemset(err_.get(), 0, sizeof(int)));
    TZ_HIP(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    mine = node_identity();
    TZ_HIP(hipIpcGetMemHandle(&h, flags_));
    mine.append(reinterpret_cast<const char *>(&h), H);
    TZ_HIP(hipIpcGetMemHandle(&h, dXr_.get()));
    mine.append(reinterpret_cast<const char *>(&h), H);
    mine.append(reinterpret_cast<const char *>(recvOff_.data()), P * sizeof(int32_t));
  } catch (const std::exception &e) {
    err = std::string("export: ") + e.what();
    mine.clear();
  }
  const std::vector<std::string> all = ctrl->allgather(mine);
  if (!err.empty()) return err;
  const std::string me = node_identity();
  try {
    TZ_CHECK(all.size() == P, "allgather returned " << all.size() << " entries");
    peerXr_.assign(P, nullptr);
    peerFlags_.assign(P, nullptr);
    peerRecvOff_.assign(P, 0);
    for (int q = 0; q < a_.size; ++q) {
      if (q == a_.rank || (sendCount_[q] == 0 && recvCount_[q] == 0)) continue;
      const std::string &blob = all[size_t(q)];
      TZ_CHECK(blob.size() == kNodeIdBytes + 2 * H + P * sizeof(int32_t),
               "rank " << q << " exported no IPC handles");
      // a handle is only meaningful on the node that exported it
      TZ_CHECK(blob.compare(0, kNodeIdBytes, me) == 0, "rank " << q << " runs on another node");
      auto open = [&](size_t k) {
        hipIpcMemHandle_t h;
        std::memcpy(&h, blob.data() + kNodeIdBytes + k * H, H);
        void *ptr = nullptr;
        TZ_HIP(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
        opened_.push_back(ptr);
        return ptr;
      };
      peerFlags_[size_t(q)] = open(0);
      if (sendCount_[q] > 0) {
        peerXr_[size_t(q)] = open(1);
        std::memcpy(&peerRecvOff_[size_t(q)],
                    blob.data() + kNodeIdBytes + 2 * H + size_t(a_.rank) * sizeof(int32_t),
                    sizeof(int32_t));
      }
    }
  } catch (const std::exception &e) {
    return std::string("map: ") + e.what();
  }
  return "";
}

std::string DistSpmv::rccl_preflight_local() {
  // the x entries my peers need, gathered and exchanged once through RCCL on a private stream
  // under a bounded wait (a hang releases spinning kernels, aborts the communicator and
  // reports), then every received entry checked
  if (!comm_) return "";
  const double limit = preflight_limit_s(20.0);
  hipStream_t s = nullptr;
  TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::string why;
  auto wait = [&]() {
    const double t0 = wtime();
    while (true) {
      const hipError_t r = hipStreamQuery(s);
      if (r == hipSuccess) return true;
      if (r != hipErrorNotReady) TZ_HIP(r);
      if (wtime() - t0 > limit) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  };
  try {
    TZ_HIP(hipMemsetAsync(dXr_.get(), 0, dXr_.bytes(), s));
    scatter(s);
    exchange(s);
    if (!wait()) {
      kern::set_abort(true);
      auto c = comm_;
      std::thread([c] { c->abort(); }).detach();
      if (!wait())
        // the abort flag cannot be cleared while something still spins, and with it set every
        // device-side wait of every later candidate gives up at once: the search would measure
        // nothing. End the run with the reason instead.
        exit_with_report(6, "RCCL preflight (spmv): the device did not drain after the "
                            "communicator abort");
      kern::set_abort(false);
      why = "exchange did not complete within " + std::to_string(int(limit)) + " s (communicator aborted)";
    } else {
      std::vector<float> xr(remoteCols_.size());
      if (!xr.empty()) dXr_.download(xr.data(), xr.size() * 4);
      size_t wrong = 0;
      for (size_t i = 0; i < xr.size(); ++i) wrong += xr[i] != x_value(remoteCols_[i]);
      if (wrong) why = std::to_string(wrong) + " wrong remote x entries";
    }
  } catch (const std::exception &e) {
    why = e.what();
  }
  (void)hipStreamDestroy(s);
  return why;
}

void DistSpmv::rccl_graph_preflight(Ctrl &ctrl) {
  // The exchange as the runtime compiles candidates (GraphBuilder: scatter, then the grouped
  // RCCL exchange), launched twice with a different local x each time, so that a graph that
  // delivers the previous launch's data fails the check. The capture mode is per process: once
  // a workload's preflight has settled it (the halo's, in a fused graph), only that mode is
  // verified here; otherwise whole-schedule capture first, then child capture. No mode works:
  // RCCL exchanges stay out of hipGraphs (their candidates run eagerly). Every rank in step.
  const double limit = preflight_limit_s(20.0);
  const std::string failEnv = std::getenv("TZ_FAIL_TRANSPORTS") ? std::getenv("TZ_FAIL_TRANSPORTS") : "";
  const bool simGraph = ("," + failEnv + ",").find(",rccl_graph_schedule,") != std::string::npos;
  std::vector<CaptureMode> modes;
  if (capture_mode_forced() || rccl_capture_settled()) modes = {rccl_capture_mode()};
  else modes = {CaptureMode::Schedule, CaptureMode::Child};
  hipStream_t s = nullptr;
  TZ_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto wait = [&]() {
    const double t0 = wtime();
    while (true) {
      const hipError_t r = hipStreamQuery(s);
      if (r == hipSuccess) return true;
      if (r != hipErrorNotReady) TZ_HIP(r);
      if (wtime() - t0 > limit) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  };
  auto upload_x = [&](int gen) {
    std::vector<float> x(xLocal_.size());
    for (size_t i = 0; i < x.size(); ++i) x[i] = xLocal_[i] + float(gen);
    if (!x.empty()) dX_.upload(x.data(), x.size() * 4);
  };
  std::vector<std::string> tried;
  bool chosen = false, hung = false;
  for (CaptureMode mode : modes) {
    std::string wrong;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    try {
      {
        GraphBuilder gb({s}, mode);
        gb.add(0, {}, [&](void *cs) {
          scatter(cs);
          exchange(cs);
        });
        graph = static_cast<hipGraph_t>(gb.finish());
      }
      TZ_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    } catch (const std::exception &e) {
      wrong = e.what(); // a capture or instantiation error: RCCL stays for eager runs
    }
    // launch only where every rank built the graph: a rank launching alone would wait for peers
    // that never join, report a hang and abort the communicator instead of trying the next mode
    double built = wrong.empty() ? 0.0 : 1.0;
    ctrl.allreduce_max(&built, 1);
    if (built != 0.0 && wrong.empty()) wrong = "capture or instantiation failed on another rank";
    try {
      for (int gen = 1; gen <= 2 && wrong.empty() && !hung; ++gen) {
        upload_x(gen);
        TZ_HIP(hipMemsetAsync(dXr_.get(), 0, dXr_.bytes(), s));
        TZ_HIP(hipGraphLaunch(exec, s));
        if (!wait()) {
          hung = true;
          break;
        }
        std::vector<float> xr(remoteCols_.size());
        if (!xr.empty()) dXr_.download(xr.data(), xr.size() * 4);
        size_t bad = 0;
        for (size_t i = 0; i < xr.size(); ++i) bad += xr[i] != x_value(remoteCols_[i]) + float(gen);
        if (simGraph && mode == CaptureMode::Schedule) bad += 1; // tests: force the fallback
        if (bad) wrong = "launch " + std::to_string(gen) + ": " + std::to_string(bad) + " wrong remote x entries";
      }
    } catch (const std::exception &e) {
      wrong = e.what(); // a capture or instantiation error: RCCL stays for eager runs
      if (!wait()) hung = true;
    }
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    double flags[2] = {hung ? 1.0 : 0.0, wrong.empty() ? 0.0 : 1.0};
    ctrl.allreduce_max(flags, 2);
    if (flags[0] != 0.0) {
      hung = true;
      break;
    }
    if (flags[1] == 0.0) {
      if (!rccl_capture_settled() && !capture_mode_forced()) set_rccl_capture_mode(mode);
      rcclCaptureNote_ = std::string(capture_mode_name(mode)) + " capture";
      if (!tried.empty()) rcclCaptureNote_ += " (" + tried.front() + ")";
      chosen = true;
      break;
    }
    tried.push_back(std::string(capture_mode_name(mode)) + " capture: " +
                    (wrong.empty() ? "wrong data on another rank" : wrong));
  }
  if (hung) {
    // a captured exchange that never completes: release spinning kernels and abort the
    // communicator as the eager preflight does; RCCL is then gone for this workload
    kern::set_abort(true);
    auto c = comm_;
    std::thread([c] { c->abort(); }).detach();
    if (!wait())
      exit_with_report(6, "RCCL graph preflight (spmv): the device did not drain after the "
                          "communicator abort");
    kern::set_abort(false);
    TZ_CHECK(a_.transport == "auto" && useIpc_ && ipcReady_,
             "SpMV RCCL transport: a captured exchange hung and there is no IPC fallback");
    comm_.reset();
    useRccl_ = false;
    rcclCaptureNote_ = "hipGraph exchange hung (communicator aborted)";
    TZ_LOG(Warn, "SpMV RCCL transport dropped: " << rcclCaptureNote_);
  } else if (!chosen) {
    rcclGraphOk_ = false;
    rcclCaptureNote_ = "eager only";
    for (const std::string &t : tried) rcclCaptureNote_ += "; " + t;
    TZ_LOG(Warn, "SpMV RCCL exchanges run eagerly only: " << rcclCaptureNote_);
  }
  upload_x(0);
  (void)hipStreamDestroy(s);
}

void DistSpmv::ipc_preflight(Ctrl *ctrl) {
  // one complete put -> wait -> release round whose arrivals are checked value by value; any
  // failure turns IPC off for every rank
  double bad = 0;
  std::string why;
  const double keep = ipcTimeoutS_;
  ipcTimeoutS_ = std::min(ipcTimeoutS_, 3.0);
  try {
    put(nullptr);
    wait_puts(nullptr);
    TZ_HIP(hipDeviceSynchronize());
  } catch (const std::exception &e) {
    bad = 1;
    why = std::string("preflight: ") + e.what();
  }
  ctrl->barrier(); // outside the try: every rank reaches it
  if (bad == 0) {
    try {
      const int e = ipc_errors();
      std::vector<float> xr(remoteCols_.size());
      if (!xr.empty()) dXr_.download(xr.data(), xr.size() * 4);
      size_t wrong = 0;
      for (size_t i = 0; i < xr.size(); ++i) wrong += xr[i] != x_value(remoteCols_[i]);
      if (e || wrong) {
        bad = 1;
        why = "preflight: " + std::to_string(e) + " wait timeout(s), " + std::to_string(wrong) +
              " wrong remote x entries";
      }
      release(nullptr);
      TZ_HIP(hipDeviceSynchronize());
    } catch (const std::exception &ex) {
      bad = 1;
      why = std::string("preflight check: ") + ex.what();
    }
  }
  ipcTimeoutS_ = keep;
  ctrl->allreduce_max(&bad, 1);
  if (bad != 0) {
    ipcReady_ = false;
    TZ_LOG(Warn, "SpMV ipc transport disabled: " << (why.empty() ? "failed on another rank" : why));
    TZ_CHECK(a_.transport != "ipc", "SpMV ipc transport requested but " << why);
  }
  ctrl->barrier();
}

void DistSpmv::put(void *stream) const {
  TZ_CHECK(ready() && useIpc_, "SpMV ipc transport not set up");
  std::vector<int> to;
  std::vector<kern::PutSeg> segs;
  for (int q = 0; q < a_.size; ++q) {
    if (q == a_.rank || sendCount_[q] == 0) continue;
    TZ_CHECK(peerXr_[size_t(q)] && peerFlags_[size_t(q)], "rank " << q << " is not IPC-mapped");
    kern::PutSeg sg;
    sg.dst = static_cast<float *>(peerXr_[size_t(q)]) + peerRecvOff_[size_t(q)];
    sg.off = sendOff_[q];
    sg.n = sendCount_[q];
    // the receiver counts my arrivals in its slot `my rank`
    sg.flag = static_cast<unsigned long long *>(peerFlags_[size_t(q)]) + a_.rank;
    segs.push_back(sg);
    to.push_back(q);
  }
  if (segs.empty()) return;
  // flow control: my put n+1 may overwrite q's remote-x entries only after q's remote product
  // of put n returned the credit (to my slot size + q)
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_) + a_.size, sent_.as<unsigned long long>(),
                 to.data(), int(to.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/1);
  kern::gather_put_signal(dX_.as<float>(), dSendIdx_.as<int32_t>(), segs.data(), int(segs.size()),
                          done_.as<unsigned int>(), stream);
}

void DistSpmv::wait_puts(void *stream) const {
  TZ_CHECK(ready() && useIpc_, "SpMV ipc transport not set up");
  std::vector<int> from;
  for (int q = 0; q < a_.size; ++q)
    if (q != a_.rank && recvCount_[q] > 0) from.push_back(q);
  kern::ipc_wait(static_cast<const unsigned long long *>(flags_), expected_.as<unsigned long long>(),
                 from.data(), int(from.size()), err_.as<int>(), ipcTimeoutS_, stream, /*lag=*/0);
}

void DistSpmv::release(void *stream) const {
  TZ_CHECK(ready() && useIpc_, "SpMV ipc transport not set up");
  std::vector<unsigned long long *> credits;
  for (int q = 0; q < a_.size; ++q)
    if (q != a_.rank && recvCount_[q] > 0)
      credits.push_back(static_cast<unsigned long long *>(peerFlags_[size_t(q)]) + a_.size + a_.rank);
  kern::ipc_signal(credits.data(), int(credits.size()), stream);
}

int DistSpmv::ipc_errors() {
  if (!useIpc_ || !err_.get()) return 0;
  int e = 0;
  TZ_HIP(hipDeviceSynchronize());
  err_.download(&e, sizeof(e));
  TZ_HIP(hipMemset(err_.get(), 0, sizeof(int)));
  return e;
}

OpPtr DistSpmv::local_op(bool accum, const std::string &p) {
  // the local product, or (kernel_choice) a ChoiceOp over the lanes-per-row kernels, the
  // CSR-stream kernel and rocSPARSE; both transports' graphs use the same op names for it
  auto self = std::const_pointer_cast<const DistSpmv>(shared_from_this());
  if (!a_.kernel_choice) return std::make_shared<SpmvLocal>(self, p + "yl", 0, accum);
  std::vector<OpPtr> ch;
  for (int w : {4, 8, 16})
    ch.push_back(std::make_shared<SpmvLocal>(self, p + "yl_w" + std::to_string(w), w, accum));
  for (int w : {1, 2, 4})
    ch.push_back(std::make_shared<SpmvLocal>(self, p + "yl_i" + std::to_string(w), kern::kSpmvIlp + w, accum));
  ch.push_back(std::make_shared<SpmvLocal>(self, p + "yl_stream", -1, accum));
  if (!a_.library.empty())
    ch.push_back(std::make_shared<SpmvLocal>(self, p + "yl_rocsparse_" + a_.library, kLibrary, accum));
  return std::make_shared<StaticChoiceOp>(p + "yl", ch);
}

std::shared_ptr<Graph> DistSpmv::form_graph_ipc(bool accum, const std::string &p) {
  // the reference's Scatter -> PostSend / PostRecv -> WaitRecv becomes put (gather straight
  // into the peers' memory) -> wait; the remote product hands the buffer back (credit)
  auto self = std::const_pointer_cast<const DistSpmv>(shared_from_this());
  auto g = std::make_shared<Graph>();
  OpPtr yl = local_op(accum, p);
  auto put = std::make_shared<SpmvPut>(self, p + "put");
  auto wait = std::make_shared<SpmvWait>(self, p + "wait");
  auto yr = std::make_shared<SpmvRemoteRelease>(self, p + "yr", accum);
  g->start_then(yl);
  g->start_then(put);
  g->then(put, wait);
  g->then(wait, yr);
  if (accum) {
    g->then(yl, yr);
    g->then_finish(yr);
  } else {
    auto y = std::make_shared<SpmvAdd>(self, p + "y");
    g->then(yl, y);
    g->then(yr, y);
    g->then_finish(y);
  }
  return g;
}

void DistSpmv::add(void *stream) const {
  kern::vector_add_f32(int(local_rows()), dYl_.as<float>(), dYr_.as<float>(), dY_.as<float>(), stream);
}

std::shared_ptr<Graph> DistSpmv::form_graph(bool accum, const std::string &p) {
  // reference SpMV CompoundOp (ops_spmv.cuh:300-436): Scatter -> PostSend/PostRecv ->
  // WaitRecv -> remote SpMV, local SpMV, VectorAdd. Here the post/wait pairs are one
  // stream-ordered RCCL exchange.
  auto self = std::const_pointer_cast<const DistSpmv>(shared_from_this());
  auto g = std::make_shared<Graph>();
  OpPtr yl = local_op(accum, p);
  auto scatter = std::make_shared<SpmvScatter>(self, p + "Pack");
  auto xchg = std::make_shared<SpmvExchange>(self, p + "exchange");
  auto yr = std::make_shared<SpmvRemote>(self, p + "yr", accum);
  g->start_then(yl);
  g->start_then(scatter);
  g->then(scatter, xchg);
  g->then(xchg, yr);
  if (accum) {
    // y = A_l x must land before y += A_r x_r
    g->then(yl, yr);
    g->then_finish(yr);
  } else {
    auto y = std::make_shared<SpmvAdd>(self, p + "y");
    g->then(yl, y);
    g->then(yr, y);
    g->then_finish(y);
  }
  return g;
}

std::shared_ptr<const Graph> DistSpmv::op_graph() {
  if (inner_) return inner_;
  const std::string &p = a_.prefix;
  const std::string &f = a_.form;
  TZ_CHECK(f == "split" || f == "accum" || f == "choice",
           "SpMV form must be split, accum or choice (got " << f << ")");
  // one transport's graph: a single form, or both forms as a ChoiceOp (accum-form op names
  // carry an extra "a_" so every op name stays unique in the expanded graph)
  auto forms = [&](bool ipc, const std::string &q) -> std::shared_ptr<Graph> {
    auto one = [&](bool accum, const std::string &r) {
      return ipc ? form_graph_ipc(accum, r) : form_graph(accum, r);
    };
    if (f != "choice") return one(f == "accum", q);
    std::vector<OpPtr> alts = {std::make_shared<StaticCompoundOp>(q + "split", one(false, q)),
                               std::make_shared<StaticCompoundOp>(q + "accum", one(true, q + "a_"))};
    auto g = std::make_shared<Graph>();
    auto c = std::make_shared<StaticChoiceOp>(q + "form", alts);
    g->start_then(c);
    g->then_finish(c);
    return g;
  };
  // graph-only builds (no setup) assume IPC can be mapped
  const bool ipc = useIpc_ && (ipcReady_ || !ready());
  const bool rccl = useRccl_ || a_.size == 1;
  TZ_CHECK(ipc || rccl, "SpMV has no transport for its x halo");
  if (ipc && rccl) {
    // the transport is a search decision too; IPC variants' op names carry "i_"
    std::vector<OpPtr> alts = {std::make_shared<StaticCompoundOp>(p + "via_rccl", forms(false, p)),
                               std::make_shared<StaticCompoundOp>(p + "via_ipc", forms(true, p + "i_"))};
    auto g = std::make_shared<Graph>();
    auto c = std::make_shared<StaticChoiceOp>(p + "xfer", alts);
    g->start_then(c);
    g->then_finish(c);
    inner_ = g;
  } else {
    inner_ = forms(ipc, ipc ? p + "i_" : p);
  }
  return inner_;
}

void DistSpmv::add_to_graph(Graph &g) {
  auto inner = op_graph();
  if (a_.compound) {
    auto c = std::make_shared<StaticCompoundOp>(a_.prefix + "spmv", inner);
    g.start_then(c);
    g.then_finish(c);
  } else {
    // splice the inner graph into g
    for (int v : inner->vertices()) {
      for (int s : inner->succs(v)) g.then(inner->op(v), inner->op(s));
    }
  }
}

} // namespace tz
