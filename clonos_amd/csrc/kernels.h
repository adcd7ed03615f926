// kernels.h -- descriptors shared by the host engine (engine.cpp) and the gfx950
// kernels (kernels.hip).  Plain structs, no HIP types.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace clg {

// ---- decode geometry ---------------------------------------------------------
// A tile is one wave's unit of decode work: a contiguous run of at most kTile bytes
// of one span, lying inside one HBM segment (or one 16 KiB window of a host-input
// staging buffer).  The tile is split into kRegions regions of kRegion bytes; each
// lane owns one region.  Coordinates inside a tile are "aligned coordinates":
// a = delta + (byte offset from the tile's first valid byte), so that abase + a is
// the byte's address and abase is 16-byte aligned.
constexpr int kRegion = 256;
constexpr int kRegions = 64;
constexpr int kTile = kRegion * kRegions;  // 16384
constexpr int kEntries = 64;               // transfer-table domain per region / per tile

struct TileDesc {
  const uint8_t* abase;  // 16-byte aligned
  uint32_t delta;        // first valid byte is abase[delta]  (delta < 16)
  uint32_t len;          // valid bytes (delta + len <= kTile)
  uint32_t span;         // owning span
  uint32_t pad;
  uint64_t span_off;     // span offset of abase[delta]
};

struct SpanDesc {
  uint32_t first_tile;
  uint32_t n_tiles;
  uint64_t len;
};

// Per-tile aggregate over tile entries e in [0, kEntries): e is the span offset of the
// first record start at/after the tile start, relative to the tile start.
// Packed u64: exit (u32, relative to the tile end; kExitErr / kExitFar sentinels) |
// cnt (u16) << 32 | wcnt (u16) << 48.
constexpr uint32_t kExitErr = 0xFFFFFFFFu;
constexpr uint32_t kExitFar = 0xFFFFFFFEu;

// Per-tile convergence info produced by the table kernel:
//   conv_entry[l]: entry offset of region l (relative to the region's first valid byte)
//                  shared by every live candidate path, or 0xFFFF if unknown;
//   conv_suffix[l]: records (low 16) and wide records (high 16) on that shared path
//                   from region l to the tile end.
struct TileConv {
  uint16_t entry[kRegions];
  uint32_t suffix[kRegions];
  uint32_t exit;       // tile exit (relative to tile end) of the shared path, or kExitErr
  uint32_t valid;      // 1 if any region converged
};

// Resolution output per tile (filled by the resolve kernel).
struct TileRes {
  uint32_t entry;      // tile-relative offset of the first record start (>= len: none)
  uint32_t limit;      // aligned coordinate where emission stops (failing record), or ~0
  uint32_t flags;      // kResTableLive: entry < kEntries and its table path is live
  uint32_t pad;
  uint64_t rec_base;   // record index of the tile's first record (span-relative)
  uint64_t wide_base;  // side-table index of the tile's first wide record (span-relative)
};
constexpr uint32_t kResTableLive = 1;

struct SpanRes {
  uint64_t n_rec;
  uint64_t n_wide;
  int32_t status;      // CLG_OK or decode error code
  int32_t err_tag;
  int64_t err_off;     // span offset of failing record
  uint64_t rec_base;   // exclusive prefix over spans (filled by the span-scan kernel)
  uint64_t wide_base;
};

struct DecodeOut {
  uint32_t* off;
  uint8_t* tag;
  int64_t* v0;
  uint32_t* w_idx;
  int32_t* w_rc;
  int64_t* w_v1;
  uint32_t* w_var_off;
  uint32_t* w_var_len;
  uint8_t* w_sub;
  uint64_t cap;
  uint64_t wcap;
};

// ---- fast decode: convergence points (decode_fast.hip) ----------------------------
// Fast-pipeline geometry: a tile's aligned coordinates [0, kTile) are split into kFOwn
// regions of kFRegion bytes (the last one takes the remainder).  Lane l < kFOwn owns
// region l; lanes kFOwn..63 compute the points of the span's NEXT tile's first kFNext
// regions (the same deterministic function that tile evaluates for itself), so a tile
// knows where its last segment must land without waiting for its neighbour.
constexpr uint32_t kFRegion = 268;  // 67 dwords: odd, so lane-strided LDS scans are conflict-free
constexpr int kFOwn = 61;
constexpr int kFNext = 3;
constexpr int kFPoints = kFOwn + kFNext;  // 64 = one wave
//
// conv[t * 64 + l] = aligned coordinate (tile t) of point l after filtering: a point is
// kept iff its candidates converged, it lies inside its tile, and it exceeds every earlier
// kept point of the same tile; kConvUnknown otherwise.
constexpr uint32_t kConvUnknown = 0xFFFFFFFFu;

// Per-lane segment [conv[l], conv[end]) parsed by k_fast_scan.  end in l+1..63 (>= kFOwn:
// a point of the next tile); kEndFail = parse failed or no point reached.
struct LaneSeg {
  uint8_t end;
  uint8_t flags;
  uint16_t far;   // end == kEndFar: the chain's next record start, bytes past the tile end
  uint32_t cnt;
  uint32_t wcnt;
};
constexpr uint8_t kEndFail = 0xFF;
// The segment passed every next-tile point (all three off the chain: a long record across
// the next tile's first region starts) and stops at a record start in the next tile instead;
// the resolve walks the next tile from there to one of its own points.
constexpr uint8_t kEndFar = 0xFE;

// Tile summary assuming the tile's entry is its first kept point f.
struct TileSum {
  uint32_t cnt, wcnt;
  uint8_t f;      // first kept own point (kEndFail: none)
  uint8_t x;      // exit: next tile's point index (0..kFNext-1) the chain lands on; kEndFail = none;
                  // kEndFar: a record start `far` bytes past the tile end
  uint16_t far;
  uint32_t pad2;
  uint64_t valid; // own lanes on the chain from f
};

struct FastRes {
  uint64_t valid;      // lanes whose segments are on the resolved path
  uint64_t rec_base;   // span-relative
  uint64_t wide_base;
};

// Device scratch the Serializable stream walker (jser_device.h) spills its handle, class
// descriptor, field and frame tables to once a stream outgrows the walker's private
// first tier.  Bump-allocated (*used reset before each decode); a walk that finds it
// full reports kJsSpill and the engine grows the arena and decodes again, so no table
// bound ever rejects a valid stream.
struct JArena {
  uint8_t* base;
  uint64_t cap;
  unsigned long long* used;
};

#ifndef CLG_FCANDS
#define CLG_FCANDS 32
#endif
constexpr int kCands = CLG_FCANDS;  // candidate entries per region (covers every fixed-layout record; <= 64)
constexpr int kJserCap = 256;  // Serializable stream-length table entries per tile

// Serializable candidates recorded where the log bytes are written (k_scatter), so the
// decode need not read the whole log to find them.  Per pool segment: hdr[s] = life << 32 |
// entries, and ent[s * cap + i] = position in the segment (low 16 bits) | code << 16, code the
// record length of the "03 AC ED 00 05" stream there (TC_STRING and flat objects that end
// inside the request's written bytes, strings well-formed) or kSideUnknown (another shape, a
// stream running past the request, or a prefix of the magic at its end: the decode verifies
// the magic and walks the stream).  A stream running past its chunk is measured on the
// request's next chunks' bytes (contiguous in the source) when the chunk says it goes on.
// `life` is the host's count of the segment's allocations (31 bits).  The chunk at a
// segment's offset 0 -- every life's first, segments filling from their start -- stamps it,
// resetting the list; a later chunk of that life with no candidate touches nothing.
// entries > cap: the list overflowed, the decode scans the segment's tiles.  Segments of
// more than 64 KiB carry no sidecar (hdr null).
constexpr uint32_t kSideUnknown = 0xFFFFu;
constexpr uint32_t kSideCapMax = 1024;  // entries per segment at most (C / 64, 64 KiB segments)
struct SideCar {
  uint64_t* hdr;
  uint32_t* ent;
  const uint8_t* pool;  // the segment pool (a tile outside it is scanned)
  uint64_t pool_bytes;
  uint32_t seg_bytes;
  uint32_t cap;
};

// Serializable stream lengths per tile, sorted by position (aligned coordinates):
// pos/len[t * kJserCap + i], n[t] entries (n > kJserCap: overflow, span falls back);
// defer[t] = 1 if the tile's scan met a "03 AC ED 00 05" pattern before the tables existed.
struct JserTabs {
  uint32_t* pos;
  uint32_t* len;
  uint32_t* n;
  uint32_t* defer;
  JArena ar;
  uint64_t* prof = nullptr;  // developer diagnostics: 16 s_memtime stamps per tile (fill 0-7, emit 8-15)
  SideCar side{};            // the write path's candidates (k_jser_fill takes a tile's table from them)
};

// Fused convergence + segment pass.  mode 0: every tile (tiles meeting a Serializable
// record are deferred); mode 1: only deferred tiles, stream-length tables filled.
int launch_fast_scan(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t* d_conv, JserTabs J,
                     uint32_t mode, LaneSeg* d_lanes, TileSum* d_sums, uint32_t* d_dbg, uint64_t* d_prof, void* stream);
int launch_jser_fill(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, JserTabs J, void* stream);
int launch_fast_resolve(const TileDesc* d_tiles, const SpanDesc* d_spans, uint32_t n_spans, uint32_t* d_conv,
                        LaneSeg* d_lanes, const TileSum* d_sums, JserTabs J, FastRes* d_fres, SpanRes* d_sres,
                        uint32_t* d_span_flags, JArena ar, void* stream);
int launch_fast_emit(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, const uint32_t* d_conv,
                     JserTabs J, const LaneSeg* d_lanes, const FastRes* d_fres, const SpanRes* d_sres,
                     const uint32_t* d_span_flags, DecodeOut out, void* stream);

// ---- fast decode (decode_fused.hip) -------------------------------------------------
// Three passes over tiles of kZTile bytes (64 regions of kZRegion bytes, one per lane):
// count (persistent grid, record chain + per-tile counts + record-start bitmaps), scan
// (record / wide bases per tile and per span), emit (SoA).  Any anomaly raises *abort and
// the host re-decodes the batch with the robust pipeline above.
constexpr uint32_t kZRegion = 128;
constexpr uint32_t kZDbgTiles = 24 + 64 * 8;  // FusedCtl.dbg: the per-tile words' start (u32 index)
constexpr uint32_t kZTile = 64 * kZRegion;  // 8192
constexpr uint32_t kZHalo = 64;             // bytes of the span's next tile staged after a tile

struct FusedCtl {
  uint64_t* st_x;     // per tile: pk_word(2, exit (span offset) the successor enters at)
  uint64_t* cnt;      // per tile: wide<<31 | records
  uint64_t* base;     // per tile: exclusive prefix of cnt inside its block of 1024 tiles
  uint64_t* boff;     // per block of 1024 tiles: exclusive prefix of the block totals
  uint64_t* bits;     // per tile: 64 x 16 B record-start bitmaps (lane l: region l)
  uint64_t* span_lo;  // per span: base at its first tile
  uint64_t* span_hi;  // per span: base past its last tile
  uint32_t* abort;    // [8]: flag, then ~(first tile) per abort reason 1..4 (4 = wait timed out)
  uint32_t* dbg;      // optional diagnostics (CLONOS_FUSED_DEBUG): [0, 16) the first aborting tile and
                      // a repair walk that gave up, [16, 24) chunk-entry reads not taken, [24, ..)
                      // the first aborting tile's lane state, then from word kZDbgTiles per tile the
                      // writer of its ex word and its entry
  uint64_t* prof;     // optional per-tile phase stamps (CLONOS_SCAN_PHASES): s_memtime x 8
  uint32_t n_tiles;
  // Serializable record lengths per tile (phase 3, k_decode_jser), sorted by position:
  // jpos/jlen[t * kZJCap + i] (aligned coordinate, record length or 0 for an invalid
  // stream), jn[t] entries.  jser = 1: the tables exist and the passes use them.
  uint32_t* jpos;
  uint32_t* jlen;
  uint32_t* jn;
  uint32_t jser;
  uint32_t jwork_cap;  // capacity of the general-walker work list
  uint32_t* jwork;     // [0]: items, [1]: overflow entries taken, then [2, 2 + cap): the items'
                       // table slots, [2 + cap, 2 + 2 cap): their tiles; with the sidecar then
                       // [2 + 2 cap]: tiles to scan, and those tiles (n_tiles words)
  uint32_t warm;    // speculative warm-up bytes before each region (| 1 << 31: not staggered by lane)
  JArena jar;       // the stream walker's spill arena (k_decode_jser_general)
  // Per-span fallback: a tile whose chain goes wrong (reasons 1-3, 5) sets span_bad[span]
  // and the count pass goes on with the next span; the host decodes the bad spans with the
  // robust pipeline, injects their counts (k_decode_inject) and re-runs scan + emit with
  // skip_bad set, so emit leaves the bad spans' records to the robust output.
  uint32_t* span_bad;
  uint32_t skip_bad;
  // Count pass: block b's chunk is tiles [chunk[b], chunk[b + 1]) (chunks of about equal
  // bytes, decode_count_chunks), or null: equal tile counts.  A batch of many small spans
  // beside a few large ones (config 4: 320-byte subpartition logs, 22 KB main logs) would
  // otherwise give a few blocks chunks of only large tiles and make them the critical path.
  const uint32_t* chunk;
  uint32_t tiny;  // pass 0 ran (k_decode_count_tiny): small whole spans are counted already
  // Chunk-boundary repair (k_decode_count files, k_decode_repair serves): ex[t] = 1 << 63 |
  // the tile's exit (span offset), 0 while unknown; rep_flag[c] = 1: chunk c needs a check;
  // ent[c] = pk_word(2, the span offset chunk c's first tile entered at) when it entered at a
  // published exit (0: it did not).  k_decode_repair compares every such entry with the true
  // exit ex[] of the tile before, after the count pass, so a chunk that took a wrong entry is
  // walked again whatever the hand-off read returned.  rep[0]: chunks served for a wrong
  // entry, rep[1]: requests filed, rep[2]: look-back checks failed (k_decode_emit; the batch
  // is decoded again), rep[3]: canonical exits found before their tile's end (published as
  // the tile end, a guess the repair checks).  All zeroed per batch.
  uint64_t* ex;
  uint8_t* rep_flag;
  uint32_t* rep;
  uint64_t* ent;
  // Test switch (CLONOS_FUSED_PERTURB): bits 15:0 are added to every chunk entry taken from a
  // published exit (and every small-path entry) -- the wrong entries the checks must catch;
  // bit 16 makes scan block 1's look-back result one record too high.  0 in production.
  uint32_t perturb;
  // 1: the one-launch scan (k_decode_scan) computed boff, and emit checks each block's
  // look-back result against its predecessor's final word (lb).  0: the three-launch scan.
  uint32_t lb_check;
  uint32_t n_spans;  // (the abort words' place in h_res)
  // Decode errors kept on the fast path: span_err[s] = the lowest span offset where a true
  // chain of span s met an invalid record (~0: none; atomicMin), and the tile holding it
  // writes the counts and start bits of the records before it.  null: off.
  uint64_t* span_err;
  // Serializable tables past kZJCap entries: entry i >= kZJCap of tile t at slot
  // n_tiles * kZJCap + jbase[t] + i - kZJCap of jpos / jlen (jovf_cap slots in all, taken
  // with jwork[1]; exhausted: abort reason 6, the host grows the arena and runs again).
  uint32_t* jbase;
  uint32_t jovf_cap;
  // The one-launch scan (phase 5, k_decode_scan): lb[0] a ticket counter, lb[1 + b] block b's
  // look-back word (pk_word state 1 and its total, then state 2 and its inclusive prefix; the
  // state is held in both halves, see decode_fused.hip); all zeroed per
  // batch.  h_res: host memory the host reads the batch's result from -- span_hi at
  // [n_spans + s], the abort words as u32 at [2 n_spans] -- written by that kernel, so no
  // read-back copy is queued (null: none).
  uint64_t* lb;
  uint64_t* h_res;
  uint32_t lean;  // batches without tables: the lean speculative walk (wide tags step one byte)
  // The write path's Serializable candidates (SideCar, below): phase 3 builds a tile's table
  // from its segment's list instead of scanning the tile (hdr null: every tile is scanned).
  SideCar side;
};
constexpr uint32_t kZAbortWords = 12;  // abort[8] rep[4] (u32), adjacent
constexpr uint32_t kZJCap = 256;  // Serializable candidates per tile in LDS (more: the overflow arena)
constexpr uint32_t kZScanBlock = 1024;  // tiles per workgroup of the offsets scan
constexpr uint32_t kZTinySpan = 1024;   // whole spans up to this many bytes: pass 0, a lane each
// abort reasons: 1 invalid record on the true chain, 2 span end, 3 exit mismatch,
// 4 wait timeout, 5 Serializable record met without tables, 6 a Serializable arena or work
// list full (the host grows it and runs again);
// abort[7] != 0: phase 3 found Serializable candidates (any tile)
// phase 0: count, 1: scan, 2: emit, 3: Serializable tables, 4: small whole spans (before 0)
// Per-span fallback: cnt[t] of every tile of bad span bad[i] := t == its first tile ?
// packed[i] (the robust decode's wide << 31 | records) : 0.
int launch_decode_inject(const SpanDesc* d_spans, const uint32_t* d_bad, const uint64_t* d_packed, uint32_t n_bad,
                         FusedCtl ctl, void* stream);
// x[i] += delta for i < n (the robust output's wide-row record indices moved into place).
int launch_add_u32(uint32_t* d_x, uint64_t n, uint32_t delta, void* stream);
// Per-span fallback, last step: bad span i's robust records (scratch rows [rbase, rbase + nrec),
// wide rows [wbase, wbase + nwide)) into the batch output at the span's bases from the re-run
// scan (ctl.span_lo), the wide rows' record indices moved by (batch base - rbase).
struct SfPlace {
  uint64_t rbase, nrec, wbase, nwide;
  uint32_t span, pad;
};
int launch_sf_place(const SfPlace* d_place, uint32_t n_bad, DecodeOut scratch, DecodeOut out, FusedCtl ctl, void* stream);
// Per-span fallback, first step (kernels.hip): bad span bad[i] with a recorded error position
// (ctl.span_err) -- the record there classified by decodeNext's full rules.  An invalid record
// (res[2 i] = its status < 0, res[2 i + 1] = its tag, as int8): the span keeps the fast run's
// records before it (span_bad cleared, its tiles past the error get no records).  Else (a
// valid record there: res[2 i] = 0) the span stays bad for the robust pipeline.
int launch_err_classify(const TileDesc* d_tiles, const SpanDesc* d_spans, const uint32_t* d_bad, uint32_t n_bad,
                        FusedCtl ctl, int32_t* d_res, JArena ar, void* stream);
int launch_decode_fused(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t n_spans,
                        FusedCtl ctl, DecodeOut out, void* stream, uint32_t phase);
// The count pass's grid for n_tiles tiles (the blocks the device keeps resident, at most one
// per tile); CLG_E_DEVICE as 0.
uint32_t decode_count_grid(bool jser, uint32_t n_tiles);

// Small batches in one launch (k_decode_small_tiles): a block per tile counts the tile from
// its predecessor's published exit, publishes its own exit and counts, sums every earlier
// tile's (look-back), emits.  Batches without Serializable tables.  Results go to `res`
// (host-mapped pinned memory or device): res[0] records, res[1] wide rows, res[2] != 0 when any
// tile failed (the host then decodes the batch the usual way), res[3 + s] span s's first record
// (spans with tiles).  agg: kZSmallAggWords zeroed words; the kernel zeroes all of agg_next for
// the next call (the host alternates two buffers, so no memset is queued).  plan (host memory,
// optional): a plan of at most kZSmallArgTiles tiles and kZSmallArgSpans spans goes in the
// launch's own arguments instead of d_tiles / d_spans, so no copy is queued before the launch.
constexpr uint32_t kZSmallSpans = 4096;     // spans per small batch at most
constexpr uint32_t kZSmallTilesMax = 4096;  // tiles per small batch at most
constexpr uint32_t kZSmallAggWords = 2 * kZSmallTilesMax;  // look-back words per buffer: counts, exits
constexpr uint32_t kZSmallArgTiles = 64, kZSmallArgSpans = 64;
struct SmallPlanArg {  // 3 KiB: with the other arguments inside the 4 KiB kernel-argument limit
  TileDesc tiles[kZSmallArgTiles];
  SpanDesc spans[kZSmallArgSpans];
};
int launch_decode_small(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans, uint32_t n_spans,
                        FusedCtl ctl, DecodeOut out, uint64_t* agg, uint64_t* agg_next, uint64_t* res, void* stream,
                        const SmallPlanArg* plan = nullptr);

// ---- gather (delta slice) -------------------------------------------------------
// A piece copies len bytes from src to out + dst; the source range lies inside one
// segment.  Pieces are produced per slice request and split at segment boundaries.
struct GatherPiece {
  const uint8_t* src;
  uint64_t dst;
  uint32_t len;
  uint32_t pad;
};

// ---- append scatter ---------------------------------------------------------------
struct ScatterChunk {
  uint8_t* dst;        // inside one segment
  uint64_t src;        // offset into the staged upload buffer
  uint32_t len;
  uint32_t life;       // causal-log chunks: the segment's life stamp (SideCar, 31 bits) | 1 << 31:
                       // the request goes on in the next chunk, its source bytes contiguous
};

// ---- device-side planning ---------------------------------------------------------
// A run of a log's physical bytes.  Its gather pieces (one per segment it touches) or
// decode tiles (one per min(segment, kTile) window) are generated on the device from the
// log's segment-index table, uploaded once per call as one concatenated array, so host
// work per call is O(requests + logs), not O(segments).
struct SegSpan {
  uint64_t segtab_off;  // first entry of the log's segment indices in the call's table
  uint32_t phys;        // first physical byte of the run
  uint32_t len;
  uint64_t dst;         // gather: output offset of the run; decode: span index
  uint32_t first;       // first piece / tile generated for the run
  uint32_t pad;
};
// Launch helpers' status: CLG_OK, or CLG_E_DEVICE with the HIP error kept (thread-local)
// for the engine's error text (take_launch_error, nullptr when none).
int launch_status(hipError_t e);
const char* take_launch_error();
int launch_expand_pieces(const SegSpan* d_spans, uint32_t n_spans, uint32_t n_pieces, const uint32_t* d_segtab,
                         const uint8_t* pool, uint32_t seg_bytes, GatherPiece* d_out, void* stream);
int launch_expand_tiles(const SegSpan* d_spans, uint32_t n_spans, uint32_t n_tiles, const uint32_t* d_segtab,
                        const uint8_t* pool, uint32_t seg_bytes, uint32_t unit, TileDesc* d_out, void* stream);
// The fast decode's set-up in one launch: n_tiles tiles expanded from the runs (as
// k_expand_tiles; 0: none), then each word range r[] copied from src or filled with val.
constexpr int kPrepRanges = 8;
struct PrepRange {
  uint32_t* dst;
  const uint32_t* src;  // null: fill
  uint64_t n;           // 32-bit words
  uint32_t val;
  uint32_t pad;
};
struct PrepArgs {
  const SegSpan* runs;
  uint32_t n_runs, n_tiles;
  const uint32_t* segtab;
  const uint8_t* pool;
  uint32_t C, U;
  TileDesc* tiles;
  uint64_t total;  // (set by the launcher)
  PrepRange r[kPrepRanges];
};
int launch_decode_prep(PrepArgs a, void* stream);

// ---- launchers (kernels.hip) -----------------------------------------------------------
// side: the causal pool's sidecar (null: no candidates recorded, e.g. in-flight log buffers)
int launch_scatter(const ScatterChunk* d_chunks, uint32_t n, const uint8_t* d_src, void* stream,
                   const SideCar* side = nullptr);
int launch_gather(const GatherPiece* d_pieces, uint32_t n, uint8_t* d_out, void* stream);
// Robust pipeline (per-byte DP transfer tables); runs only on spans whose flag is set
// (d_span_flags == nullptr: all spans).
int launch_decode_tables(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans,
                         uint64_t* d_agg, TileConv* d_conv, const uint32_t* d_span_flags, JArena ar, void* stream);
int launch_decode_resolve(const TileDesc* d_tiles, const SpanDesc* d_spans, uint32_t n_spans,
                          const uint64_t* d_agg, const TileConv* d_conv, TileRes* d_tres,
                          SpanRes* d_sres, const uint32_t* d_span_flags, JArena ar, void* stream);
int launch_decode_spanscan(SpanRes* d_sres, uint32_t n_spans, uint64_t* d_totals, void* stream);
int launch_decode_emit(const TileDesc* d_tiles, uint32_t n_tiles, const SpanDesc* d_spans,
                       const TileConv* d_conv, const TileRes* d_tres, const SpanRes* d_sres,
                       const uint32_t* d_span_flags, DecodeOut out, JArena ar, void* stream);


// ---- batched encode (encode.hip) -------------------------------------------------
struct EncodeIn {  // device pointers, the decode's SoA layout (clg_decoded)
  const uint8_t* tag;
  const int64_t* v0;
  const uint32_t* w_idx;
  const int32_t* w_rc;
  const int64_t* w_v1;
  const uint32_t* w_var_off;  // into var
  const uint32_t* w_var_len;
  const uint8_t* w_sub;
  const uint8_t* var;
  uint64_t n, n_wide;
};
// phase 0: wide prefix per block (wsum -> wbase, nb + 1), bytes per block (bsum -> bbase,
// nb + 1), *bad = lowest invalid record; phase 1: write.  nb = ceil(n / 1024).
int launch_encode(const EncodeIn& in, uint32_t* d_wsum, uint64_t* d_wbase, uint64_t* d_bsum, uint64_t* d_bbase,
                  uint32_t* d_bad, uint8_t* d_out, uint32_t phase, void* stream);

// ---- replay preparation: subpartition recovery buffers ----------------------------
// A recovery buffer may hold BufferBuilt determinants only (ReplayingState.java:172-177),
// which are 5 bytes each, so record k of a well-formed buffer starts at 5k: no chain walk.
struct BufSpan {
  const uint8_t* src;  // device bytes
  uint64_t len;
  uint64_t out_base;   // first index in the sizes array
};
struct BufChunk {      // records [k0, k1) of span `span`
  uint32_t span;
  uint32_t pad;
  uint64_t k0, k1;
};
// first_bad[s] = lowest k whose record is not a complete BufferBuilt (init ~0).
int launch_bufsizes(const BufChunk* d_chunks, uint32_t n_chunks, const BufSpan* d_spans, int32_t* d_sizes,
                    uint64_t* d_first_bad, void* stream);
// Per span: the count of valid sizes, and the status SubpartitionRecoveryThread.run hits at
// record first_bad (decodeNext's error, or CLG_E_NOT_BUFFER_BUILT for a valid other record).
int launch_bufsizes_classify(const BufSpan* d_spans, uint32_t n_spans, const uint64_t* d_first_bad,
                             uint64_t* d_count, int32_t* d_status, int64_t* d_err_off, int32_t* d_err_tag,
                             JArena ar, void* stream);

}  // namespace clg
