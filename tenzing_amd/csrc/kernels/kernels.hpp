// Host-side launch API of the hand-written gfx950 kernels (implemented in *.hip).
// All launches are asynchronous on the given hipStream_t (passed as void* so host-only
// translation units need no HIP headers) and never allocate or synchronize, so they can be
// captured into hipGraphs.
#pragma once

#include <cstdint>
#include <vector>
#include <string>

namespace tz {
namespace kern {

/// A 4-D box inside a pitched array, copied to/from a dense buffer.
/// The box is `n3 x n2 x n1` rows of `len` contiguous elements; row (i1,i2,i3) starts at
/// element `grid_off + i1*s1 + i2*s2 + i3*s3` of the array; the buffer is dense
/// ((i3*n2 + i2)*n1 + i1)*len + x. For the XYZQ halo layout rows are x-runs and
/// (i1,i2,i3) = (y,z,q); for QXYZ rows are (q,x)-runs and (i1,i2,i3) = (y,z,1).
struct BoxDesc {
  double *buf = nullptr;
  int64_t grid_off = 0;
  int64_t s1 = 0, s2 = 0, s3 = 0;
  int32_t len = 0, n1 = 0, n2 = 0, n3 = 0;
  /// unpack only: elements of row padding before / after each grid row that the writes may
  /// also cover (their values are undefined), so that short rows (x ghost runs of 9 doubles)
  /// become whole 16-B-aligned sectors written with 16-B stores; 0, 0: exactly the box
  int32_t lead = 0, trail = 0;
};

constexpr int kMaxBoxes = 32;

/// launch tuning of the box kernels (process-wide; measured defaults)
struct BoxTuning {
  // pack / unpack: items per lane the grid is sized for; 4 or 8 keep that many loads in flight,
  // 1-3 keep one in flight. 3 packs and unpacks 2 % faster than 4 in pipeline context
  // (scripts/ktune.py --unrolls, profiles/archive/r2_move_shape/ktune_unrolls*.jsonl); 8 is slower
  int unroll = 3;
  bool nt_pack = true;    // non-temporal grid loads in pack: -27 % pack time in pipeline context
  // non-temporal ghost stores in unpack: the ghosts are not read again within the exchange.
  // Round 1 measured +5 % on the one-rank pack -> copy -> unpack chain; the receive-buffer
  // unpack of the multi-rank exchange gains 7-8 % (2 loopback ranks, 0.228-0.239 -> 0.210-0.218
  // ms, scripts/nt_multi_ab.sh, profiles/archive/r2_nt/)
  bool nt_unpack = true;
  int max_blocks = 4096;  // cap per box (grid-stride beyond)
  // cap per box of the signalling put kernels, whose stores cross xGMI: one link moves ~77 GB/s per direction, which 64 blocks of posted 16-B
  // stores cover with a wide margin, while thousands of blocks stalled on a link would hold the
  // CU slots that the concurrent local moves, relay kernels and unpacks need
  int put_max_blocks = 64;
  // box_move (direct transfers): plain source loads and non-temporal ghost stores. The ghosts
  // are written once per exchange and nobody reads them inside it, so streaming them past the
  // caches leaves L2 / Infinity Cache to the interior slabs, which every exchange reads again:
  // 47.7 -> 44.4 us for the 26-direction move at 512^3 x 3 (scripts/move_ab.py; non-temporal
  // loads plus stores: 57.7 us).
  bool nt_move = false;
  bool nt_move_store = true;
  // box_move (direct transfers): items in flight per lane (1, 2 or 4) and
  // items per lane the grid is sized for (>= in flight; the lane loops over them). One in
  // flight, two per lane (twice the workgroups of 4 x 4) moves the 26 directions at 512^3 x 3
  // in 43.5 us against 44.1 us, the best of 10 shapes (scripts/move_ab.py --blocks,
  // profiles/archive/r2_move_shape/)
  int move_unroll = 1;
  int move_items = 2;
  int xcd_remap = 0; // box_move block order: 0 round-robin, 1 one contiguous range per XCD,
                     // 2 every box split into 8 contiguous per-XCD shares
  // moves of rows that start one element past a 16-B boundary peel that element and move the
  // rest with 16-B accesses (false: 8-B accesses throughout; XYZQ row-start layout, 26
  // directions: 92.0 -> 88.8 us, profiles/r5_roof/)
  bool peel_moves = true;
  // unpack boxes with lead / trail (BoxDesc) write their widened rows with 16-B stores (false:
  // exactly the box; the 26-direction unpack 66 -> 37 us, profiles/r5_unpack/)
  bool widen_unpack = true;
};
BoxTuning &box_tuning();
/// set BoxTuning::xcd_remap; throws std::invalid_argument unless mode is 0, 1 or 2
void set_xcd_remap(int mode);

/// A box-to-box move between two arrays of the SAME pitched layout: element (x,i1,i2,i3) of
/// the box at `src + src_off` goes to the same element of the box at `dst + dst_off`
/// (strides s1..s3, rows of `len`). This is the pack-free "direct" halo transfer: interior
/// slab -> ghost region of the neighbour's grid (own grid for self-neighbours, an IPC-mapped
/// peer grid over xGMI otherwise).
struct MoveDesc {
  const double *src = nullptr;
  double *dst = nullptr;
  int64_t src_off = 0, dst_off = 0;
  int64_t s1 = 0, s2 = 0, s3 = 0;
  int32_t len = 0, n1 = 0, n2 = 0, n3 = 0;
  /// row pair (self-wrap of the x axis in one array, src == dst): every row also moves its
  /// run [src - (dst_off - src_off) - ... ] back the other way. With delta = dst_off - src_off,
  /// row element e = src_off + row: [e, e + len) -> [e + delta, ...) AND
  /// [e + len + delta, e + 2 len + delta) -> [e + len, e + 2 len) -- the +x and -x boxes of one
  /// (dy, dz) moved by one lane per row, so that a row's ghost and source runs that share a
  /// cache line (x = 0 at the row start) are read and written while the line is in L2.
  /// At most kMaxPairLen elements per run.
  bool pair = false;
};
constexpr int kMaxPairLen = 8;
/// up to kMaxBoxes moves in ONE launch
void box_move_many(const MoveDesc *d, int n, void *stream);

/// Shape-matched roof probe of a move: whole 128-B lines of a pitched array, rows of `lines`
/// lines at `off` (elements, a multiple of 16) with strides s1..s3 (multiples of 16), read
/// (mode 0), written (mode 1) or read and written back by the same lane (mode 2), with full
/// 16-B accesses and the same flat indexing as the move. One launch for all boxes: the time of
/// touching exactly the lines a move touches, at the best access shape.
struct LineBox {
  double *base = nullptr;
  int64_t off = 0, s1 = 0, s2 = 0, s3 = 0;
  int32_t lines = 0, n1 = 0, n2 = 0, n3 = 0;
  /// 0 read, 1 write, 2 read + write back, 3 line-to-line copy to dst_base + dst_off (the
  /// move's own shape: each lane loads 16 B of a source line and stores them to its target line)
  int mode = 0;
  double *dst_base = nullptr;
  int64_t dst_off = 0;
};
/// variants: 0 one item in flight per lane + non-temporal stores, 1 four in flight + nt,
/// 2 one + plain stores, 3 four + plain
constexpr int kLineRoofVariants = 4;
void line_roof(const LineBox *boxes, int n, void *stream, int variant = 0);
/// the line boxes a batch of moves reads and writes (a move's rows at one intra-line alignment:
/// every row covers the same number of lines). `copies`: a move whose source and destination
/// rows cover the same number of lines becomes one mode-3 box (line-to-line copy, the move's
/// shape); otherwise reads and writes are separate boxes. Lines read and written by the same
/// rows become mode-2 boxes.
std::vector<LineBox> line_boxes(const MoveDesc *moves, int n, bool copies = true);
/// how box_move_many would move each box (no launch): "vec16", "vec8", "peeled", "pair" or
/// "empty"
std::vector<std::string> move_kinds(const MoveDesc *moves, int n);

/// Completion signal of a move whose destination is another rank's memory (IPC peer put):
/// when the last block of box i has stored its part, it makes every store of the box visible
/// at system scope and adds 1 to `flag[i]` (a counter in the receiver's uncached memory).
/// `done` holds one zero-initialized block counter per box (self-resetting).
struct MoveSignal {
  unsigned int *done = nullptr;
  unsigned long long *flag[kMaxBoxes] = {};
  /// store mode (flags in host memory, where a GPU read-modify-write would need PCIe
  /// AtomicOps): box k's flag has one writer, this one, so instead of adding 1 it stores
  /// ++count[k] (count: device memory, one counter per box, owned by the caller) with a
  /// system-scope release store. Boxes not in `store_mask` add 1 as usual.
  unsigned long long *count = nullptr;
  uint64_t store_mask = 0;
  /// workgroups per box at most (0: BoxTuning::put_max_blocks)
  int max_blocks = 0;
};
void box_move_many_signal(const MoveDesc *d, int n, const MoveSignal &sig, void *stream);
/// pack boxes of `grid` into their (possibly peer-mapped) dense buffers and signal each box's
/// completion like box_move_many_signal (IPC put into a neighbour's receive buffer)
void box_pack_many_signal(double *grid, const BoxDesc *d, int n, const MoveSignal &sig,
                          void *stream);

/// Device-side counter wait for IPC puts: for each of the `n` slots, spin (system-scope acquire
/// loads, s_sleep back-off) until `arrive[slot]` reaches expected[slot] + 1 - lag, then bump
/// expected[slot] and, if `signal` is given, add 1 to signal[k] (system scope, release).
/// lag 0: receiver waits for this round's arrival; lag 1: sender waits for the credit of its
/// previous put. A wait longer than `timeout_s` sets *err = 1 and gives up, so a lost peer
/// cannot hang the GPU.
void ipc_wait(const unsigned long long *arrive, unsigned long long *expected, const int *slots,
              int n, int *err, double timeout_s, void *stream, int lag = 0,
              unsigned long long *const *signal = nullptr);
/// add 1 to each of `n` (peer) counters, system scope, after the stream's prior work. With
/// `count` (device memory, n counters): store ++count[k] instead (single-writer counters in
/// host memory, no PCIe atomics; see MoveSignal::count)
void ipc_signal(unsigned long long *const *signal, int n, void *stream,
                unsigned long long *count = nullptr);

/// pack (grid -> buf) or unpack (buf -> grid) one box
void box_copy(double *grid, const BoxDesc &d, bool unpack, void *stream);
/// pack/unpack up to kMaxBoxes boxes in ONE launch (fused multi-face halo pack/unpack)
void box_copy_many(double *grid, const BoxDesc *d, int n, bool unpack, void *stream);

/// dst = src, `bytes` (16-B aligned pointers; the transport copy of self-neighbour exchanges)
void copy_bytes(void *dst, const void *src, size_t bytes, void *stream);
struct CopyDesc {
  void *dst = nullptr;
  const void *src = nullptr;
  size_t bytes = 0; // multiple of 16, 16-B aligned pointers
};
/// up to kMaxBoxes copies in one launch
void copy_many(const CopyDesc *d, int n, void *stream);

/// y[r] = sum_j A[r,j] x[j] for CSR A (f32 values, i32 indices). `lanesPerRow` in {1,2,4,8,16,32,64}
/// (0 = 8), or -1 for the CSR-stream kernel (block-contiguous nnz streaming + LDS segmented
/// reduction). When `accumulate`, y[r] += ... instead. lanesPerRow = kSpmvIlp + W (W = 1, 2, 4):
/// the ILP kernel (every lane issues 16 / W column loads, then the value loads and x gathers,
/// before using any).
constexpr int kSpmvIlp = 1000;
void csr_spmv(int nRows, const int32_t *rowPtr, const int32_t *colInd, const float *val,
              const float *x, float *y, int lanesPerRow, bool accumulate, void *stream);
/// A CSR SpMV for box_move_spmv: y = A x (accumulate: y += A x) with the ILP kernel
/// (lanes = kSpmvIlp + W, W in {1, 2, 4})
struct SpmvJob {
  int nRows = 0;
  const int32_t *rowPtr = nullptr, *colInd = nullptr;
  const float *val = nullptr, *x = nullptr;
  float *y = nullptr;
  int lanes = kSpmvIlp + 4;
  bool accumulate = false;
};
/// Horizontal fusion: up to kMaxBoxes direct moves (as box_move_many, XCD remap 0) and one
/// SpMV in ONE launch. The SpMV's workgroups are spread evenly among the move's, so both run
/// at once from the first wave on, with no fork or join between two streams: the SpMV's L2
/// gathers fill the issue slots the move's HBM stream leaves idle (one GPU, 512^3 halo +
/// 150,000-row SpMV: 54.5 us one after the other, 49.2-49.8 us on two free-running streams,
/// scripts/coexec_probe.py)
void box_move_spmv(const MoveDesc *moves, int n, const SpmvJob &job, void *stream);
/// dst[i] = src[idx[i]]
void gather_f32(int n, const float *src, const int32_t *idx, float *dst, void *stream);
/// one peer's part of an IPC put of the SpMV x halo: dst[i] = src[idx[off + i]], i < n, then
/// *flag += 1 (system scope) once the whole segment is visible
struct PutSeg {
  float *dst = nullptr;
  int32_t off = 0, n = 0;
  unsigned long long *flag = nullptr;
};
constexpr int kMaxPutPeers = 64;
/// all peers' segments in one launch; `done` holds one zeroed completion counter per segment
void gather_put_signal(const float *src, const int32_t *idx, const PutSeg *segs, int nseg,
                       unsigned int *done, void *stream);
/// y = a + b (f32, vectorized)
void vector_add_f32(int n, const float *a, const float *b, float *y, void *stream);
/// y += alpha * x (f64)
void axpy_f64(int64_t n, double alpha, const double *x, double *y, void *stream);
/// fill a[i] = base + scale * i (f64) — deterministic test patterns
void iota_f64(int64_t n, double base, double scale, double *a, void *stream);
/// empty kernel (launch-overhead probes, reference test/test_gpu_graph.cu:10)
void empty(void *stream);
/// spin for `ticks` of the constant-rate wall clock (synthetic device work for scheduling tests)
void busy_wait(int64_t ticks, int blocks, void *stream);

/// Process-wide device abort flag (host-coherent memory, allocated on first use). Every kernel
/// that spins (IPC arrival and credit waits, busy_wait) polls it and gives up once it is set,
/// so the runtime watchdog can drain a hung schedule's device work without killing the process.
/// The pointer is a kernel argument (hipGraph captures keep it valid: it is never freed).
const int *abort_flag();
/// host side: set or clear the flag (vector stores from the host; the kernels only load it)
void set_abort(bool on);
bool abort_set();

/// A box of the halo grid for the 7-point stencil (see stencil_kernels.hip). Element (i, y, z,
/// o) of the box is at base + o*so + z*sz + y*sy + i, for i < row (a contiguous run), y < ny,
/// z < nz, o < nouter; its x neighbours are +-xs away. The box must have a one-cell apron of
/// valid memory (ghosts) on every side.
struct StencilBox {
  const double *in = nullptr;
  double *out = nullptr;
  int64_t base = 0, sy = 0, sz = 0, so = 0;
  int32_t row = 0, ny = 0, nz = 0, nouter = 1, xs = 1;
  // elements at the start / end of every row that are neither stored nor read beyond: a box
  // can keep an aligned row (16-B accesses) while excluding its first / last x cells (the
  // ghost-free interior); the masked elements then need no apron on that side
  int32_t m0 = 0, m1 = 0;
  double c0 = 0.4, c1 = 0.1;
};
/// stencil launch shape: rows per workgroup tile (4, 8, 16) and planes per z chunk (32, 64)
struct StencilTuning {
  int ty = 16; // 64 x 16 tiles (scripts/stencil_bench.py)
  // 64-plane chunks with the tiles in XCD-contiguous order (below): 512^3 x 3, interleaved
  // A/B in one process, QXYZ 1538 us / XYZQ 1483 us, against 1569-1573 / 1566 us for the best
  // hardware-order tiling (16-plane chunks, whose 4x the workgroups had beaten 64-plane ones in
  // the hardware order) and 1605 / 1589 us for torch's copy of the padded grid
  // (profiles/r6_stencil/)
  int zc = 64;
  int pf = 1;  // planes in flight beyond z + 1 (1 or 2)
  bool db = true; // double-buffered LDS tile (one barrier per plane instead of two)
  // tiles in XCD-contiguous order (each XCD a contiguous range of tiles, so a tile's row aprons
  // come from its own L2; FETCH_SIZE -8 %) instead of the hardware's round-robin over the 8 XCDs
  bool xcd_tiles = true;
};
StencilTuning &stencil_tuning();
/// out = c0 * in + c1 * (sum of the 6 face neighbours) over the box; `lds`: 2.5-D LDS-tiled
/// kernel, else neighbours straight from global memory (both march z with a register queue)
void stencil7(const StencilBox &b, bool lds, void *stream);
/// a box one or a few cells thick (the boundary shell) goes to a one-thread-per-element kernel
bool stencil_thin(const StencilBox &b);
/// several thin boxes in one launch
void stencil7_thin_many(const StencilBox *b, int n, void *stream);

/// Halo grid geometry for init / verification kernels.
struct HaloGeom {
  int32_t order = 0; // 0 = XYZQ (x fastest, q slowest, x-padded rows), 1 = QXYZ
  int64_t xoff = 0, sy = 0, sz = 0, sq = 0; // XYZQ strides (elements)
  int32_t nx = 0, ny = 0, nz = 0, nq = 0, g = 0;
  int32_t cx = 0, cy = 0, cz = 0, px = 1, py = 1, pz = 1;
  int32_t neighbors = 6; // which ghost regions an exchange fills (6 faces, 26 all)
  int32_t gen = 0;       // generation 0..3: shifts every value, so data left over from an
                         // earlier exchange of another generation fails the check
};
/// interior = encoded global coordinate, ghosts = -1
void halo_init(double *grid, const HaloGeom &g, void *stream);
/// count elements that differ from what a completed exchange must leave; result in *count
void halo_check(const double *grid, const HaloGeom &g, unsigned long long *count, void *stream);
/// stencil mode: count interior cells of `out` that differ from the 7-point stencil (default
/// coefficients) of the field halo_init writes (global coordinates, periodic)
void stencil_check(const double *out, const HaloGeom &g, unsigned long long *count, void *stream);

} // namespace kern
} // namespace tz
