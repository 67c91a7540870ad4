/*
 * metalhuffman.h -- C-ABI of the MI355X-native Huffman block decoder.
 *
 * Drop-in boundary for the per-frame decode path of mdejong/MetalHuffman.
 * The reference binds five buffers to its Metal fragment shaders
 * (Shared/AAPLRenderer.m:1233-1253, slot enum Shared/AAPLShaderTypes.h:32-38):
 *   [0] blockStartBitOffsets  u32[NB]             (AAPLRenderer.m:1237, :863-864, :672-685)
 *   [1] huffBuff              u8[codes + 2 pad]   (AAPLRenderer.m:1243, :576-585)
 *   [2] huffSymbolTable1      HuffLookupSymbol[256] (AAPLRenderer.m:1247, :657)
 *   [3] huffSymbolTable2      HuffLookupSymbol[(k+1)*256] (AAPLRenderer.m:1250, :660)
 *   [4] dims uniform          {u16 width, height, blockWidth, blockHeight}
 *                             (AAPLShaderTypes.h:89-95, AAPLRenderer.m:1253, :768-775)
 * mh_decode() takes exactly those buffers (device pointers) and replaces the five
 * huffFragmentShaderB8W12/B8W16 passes, the 16-slice blit and the
 * cropAndGrayscaleFromTexturesFragmentShader reorder (AAPLShaders.metal:127-518,
 * AAPLRenderer.m:1192-1678) with one kernel launch that writes the W x H 8-bit
 * raster directly. The decoded value is the reference output texture's B byte.
 *
 * The producer side (mh_encode_*, mh_build_tables, ...) mirrors the reference's
 * HuffmanUtil statics / Huffman ObjC facade (Shared/HuffmanUtil.hpp:22-100,
 * Shared/Huffman.h:9-77) without module state: every call is reentrant.
 *
 * Conventions: plain pointers and sizes; `stream` is a hipStream_t (NULL = the
 * default stream); device pointers are marked d_. The library never allocates
 * on a decode call; tables are read-only during a decode. Every entry point
 * returns MH_OK (0) or a negative MH_ERR_* code; decode calls never modify the
 * output for a valid stream.
 */
#ifndef METALHUFFMAN_H
#define METALHUFFMAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_VERSION_MAJOR 0
#define MH_VERSION_MINOR 1

/* --- status codes (the reference only asserts: HuffmanEncoder.cpp:131,
 *     AAPLRenderer.m:199,215,721) --------------------------------------- */
#define MH_OK 0
#define MH_ERR_INVALID_ARG (-1)   /* NULL pointer, zero size, bad flags          */
#define MH_ERR_DIMS (-2)          /* dims inconsistent or above the u16 limits   */
#define MH_ERR_CODE_TOO_LONG (-3) /* Huffman depth > 16 (ref: assert codei < 16) */
#define MH_ERR_CAPACITY (-4)      /* caller buffer too small                     */
#define MH_ERR_TABLE (-5)         /* table2 smaller than 256 or not 256-aligned  */
#define MH_ERR_ALIGN (-6)         /* codes not 16-byte aligned / pitch % 8 != 0  */
#define MH_ERR_HIP (-7)           /* HIP runtime error (launch / no device)      */
#define MH_ERR_EMPTY (-8)         /* no symbols to encode                        */

/* --- constants (Shared/AAPLShaderTypes.h:109-123) --------------------- */
#define MH_BLOCK_DIM 8           /* HUFF_BLOCK_DIM                              */
#define MH_TABLE1_NUM_BITS 8     /* HUFF_TABLE1_NUM_BITS                        */
#define MH_TABLE2_NUM_BITS 8     /* HUFF_TABLE2_NUM_BITS                        */
#define MH_TABLE1_SIZE 256       /* HUFF_TABLE1_SIZE                            */
#define MH_TABLE2_SIZE 256       /* HUFF_TABLE2_SIZE (entries per subtable)     */
#define MH_TABLE2_MAX_ENTRIES (257 * 256)
#define MH_MAX_DIM 65535         /* u16 fields of the dims uniform              */
#define MH_CODES_PAD 4           /* zero bytes after the payload: 2 from the
                                    encoder (HuffmanEncoder.cpp:377-378) + 2 from
                                    the renderer (AAPLRenderer.m:576-585)       */

/* decode flags */
#define MH_FLAG_NO_DELTA 0x1u    /* IMPL_DELTAS_BEFORE_HUFF_ENCODING off
                                    (AAPLShaders.metal:263-265): emit symbols raw */
#define MH_FLAG_LANE_PAIRS 0x2u  /* diagnostic only: mh_decode accepts and ignores
                                    it (the default kernels decode; round 5 briefly
                                    returned MH_ERR_INVALID_ARG). The lane-pair kernel
                                    (each block on two lanes -- one from the block
                                    start, one speculatively from its middle bit,
                                    re-synchronised through ds_bpermute; same output;
                                    3.5x slower) is in the
                                    diagnostic library libmh_diag_lanepairs.so, whose
                                    mh_diag_decode_lanepairs takes mh_decode's
                                    arguments */
#define MH_FLAG_ANY_ORDER 0x4u   /* the launch may start before earlier work on
                                    the stream has finished (the AQL dispatch packet
                                    goes out without its barrier bit, HIP's
                                    hipExtAnyOrderLaunch). The caller guarantees that
                                    nothing still running on the stream writes this
                                    call's inputs or touches its output -- e.g. a run
                                    of decodes of resident frames into distinct
                                    rasters, the first of them launched without the
                                    flag. Later work on the stream still waits for it.
                                    Same output. On gfx950 the dispatches still run
                                    one after another (scripts/micro/any_order_probe
                                    .hip); the flag trims ~0.1-0.2 us of the gap
                                    between them */

/* Shared/HuffmanLookupSymbol.h:7-10: 2-byte entry. In T1, bitWidth == 0 marks
 * an escape whose `symbol` is the T2 subtable index (HuffmanUtil.cpp:639-646). */
typedef struct {
  uint8_t symbol;
  uint8_t bitWidth;
} mh_lookup_symbol;

/* Shared/AAPLShaderTypes.h:89-95 RenderTargetDimensionsAndBlockDimensionsUniform,
 * widened to u32 (values must still fit the reference's u16 fields). */
typedef struct {
  uint32_t width;
  uint32_t height;
  uint32_t block_width;  /* ceil(width / 8)  (AAPLRenderer.m:753-761) */
  uint32_t block_height; /* ceil(height / 8) */
} mh_dims;

/* One frame, or a batch of frames that share one table pair and one size.
 * Frame f's block offsets are d_block_offsets[f*NB .. f*NB+NB) (bit offsets
 * relative to frame f's first code byte); its code bytes start at
 * d_codes + frame_code_offsets[f] (16-byte aligned). */
typedef struct {
  const uint32_t *d_block_offsets;        /* slot [0], u32[n_frames * NB]      */
  const uint8_t *d_codes;                 /* slot [1], 16-byte aligned          */
  uint64_t codes_bytes;                   /* bytes readable at d_codes          */
  const uint64_t *d_frame_code_offsets;   /* u64[n_frames + 1], or NULL when
                                             n_frames == 1 (frame = whole buf) */
  const mh_lookup_symbol *d_table1;       /* slot [2], 256 entries              */
  const mh_lookup_symbol *d_table2;       /* slot [3], table2_entries entries   */
  uint32_t table2_entries;                /* (k+1)*256, k = #subtables          */
  const uint16_t *d_lut;                  /* optional: mh_prepare_lut() output,
                                             NULL = derive it inside the kernel */
  const uint8_t *d_block_init;            /* optional u8[n_frames*NB]: per-block
                                             initial prev symbol
                                             (IMPL_DELTAS_AND_INIT_ZERO_DELTA_...,
                                             AAPLRenderer.m:449-473,
                                             AAPLShaders.metal:324); NULL = 0  */
  mh_dims dims;                           /* slot [4]                           */
  uint32_t n_frames;
  uint32_t flags;                         /* MH_FLAG_*                          */
} mh_frame;

/* ---------------------------------------------------------------------- */
/* GPU decode (the hot path).                                              */

/* Decode n_frames frames into d_out: frame f, row y starts at
 * d_out + f*out_frame_stride + y*out_pitch. round_up(W, 8) bytes of each row
 * y < H are written (the kernel stores whole 8-pixel block rows, so a right-edge
 * block also writes the padding between W and round_up(W, 8)); the rest of the
 * pitch and rows >= H are not touched. out_pitch must be a multiple of 8 and
 * >= W (hence >= round_up(W, 8): rows never overlap).
 * Asynchronous on `stream`; one kernel launch. */
int mh_decode(const mh_frame *frame, uint8_t *d_out, size_t out_pitch,
              size_t out_frame_stride, void *stream);

/* Debug mode of the decode contract: walks every block of
 * `frame` exactly as mh_decode does and writes, per frame f, u32 d_report[4f..4f+3]:
 *   [0] zero-width lookups (windows no code matches -- the reference's {0,0}
 *       entry, HuffmanUtil.cpp:550-556, which repeats prev without advancing),
 *   [1] T1 escapes to a subtable at or past table2_entries (table index > k),
 *   [2] blocks whose 64 codes do not end at the next block's offset
 *       (a frame's last block is not checked),
 *   [3] the first such block (frame relative), or 0xFFFFFFFF.
 * Never writes the raster; valid reference streams report 0, 0, 0, 0xFFFFFFFF.
 * Asynchronous on `stream`. */
int mh_check(const mh_frame *frame, uint32_t *d_report, void *stream);

/* Bytes needed for the derived lookup table mh_prepare_lut() writes. */
size_t mh_lut_bytes(void);

/* Derive the decoder's 2^MH_LUT_BITS-entry first-level table from T1/T2 on the
 * device (one small kernel). Rebuild only when the tables change, exactly as
 * the reference builds T1/T2 once (AAPLRenderer.m:608). The buffer is opaque:
 * write it only through mh_prepare_lut or mh_build_tables_device -- besides the
 * entries it carries facts derived from them (longest / shortest code, whether
 * the code is the identity 8-bit code) that the decode kernels act on. */
int mh_prepare_lut(const mh_lookup_symbol *d_table1, const mh_lookup_symbol *d_table2,
                   uint32_t table2_entries, uint16_t *d_lut, void *stream);

/* Number of LUT index bits used by the kernel (first-level lookup width). */
int mh_lut_bits(void);

/* GPU-side table build from the 256-byte canonical header (the device twin of
 * mh_build_tables: HuffmanUtil.cpp:270-310 parseCanonicalHeader + :338-667
 * generateSplitLookupTables 8/8). Writes T1 (256 entries), T2 through its full
 * MH_TABLE2_MAX_ENTRIES capacity (zero beyond the (k+1)*256 used entries, so
 * mh_decode may be given table2_entries = MH_TABLE2_MAX_ENTRIES), the used entry
 * count to *d_table2_entries, and -- when d_lut is non-NULL -- the prepared
 * table (mh_prepare_lut). d_status (optional, device int32): MH_OK, or
 * MH_ERR_CODE_TOO_LONG / MH_ERR_TABLE (lengths that are not a prefix code), in
 * which case the tables are left zero. All pointers are device pointers;
 * asynchronous on `stream`. Lets a multi-GPU job broadcast 256 bytes. */
int mh_build_tables_device(const uint8_t *d_canon_header, mh_lookup_symbol *d_table1,
                           mh_lookup_symbol *d_table2, uint32_t *d_table2_entries,
                           uint16_t *d_lut, int32_t *d_status, void *stream);

/* ---------------------------------------------------------------------- */
/* GPU encoder (the producer side on the device; output byte-identical to   */
/* mh_encode_frame: HuffmanEncoder.cpp:310-381, HuffmanUtil.cpp:1051-1131,  */
/* AAPLRenderer.m:374-688).                                                 */

/* Device workspace mh_encode_frame_device / _async need for a width x height
 * frame (the larger figure, the synchronous call's). */
size_t mh_encode_workspace_bytes(uint32_t width, uint32_t height);

/* Encode the device frame d_gray (W x H bytes, row stride W) without a host
 * synchronisation: block split, deltas (unless MH_FLAG_NO_DELTA) and histogram,
 * the reference's Huffman tree (HuffmanEncoder.cpp:29-145, same tie-breaking as
 * mh_code_lengths) and canonical codes on one workgroup, block offsets (a prefix
 * sum of per-block bit lengths) and MSB-first bit packing, all on `stream`.
 * Writes d_canon_header (device u8[256]), d_codes (4-byte aligned; the byte
 * count is payload + MH_CODES_PAD zero bytes), *d_codes_len (device u64,
 * optional), d_block_offsets (u32[NB]) and, if non-NULL, d_block_init (u8[NB],
 * the IMPL_DELTAS_AND_INIT_ZERO_DELTA variant). *d_status (device int32,
 * optional) becomes MH_OK, MH_ERR_EMPTY, MH_ERR_CODE_TOO_LONG (depth > 16) or
 * MH_ERR_CAPACITY (round_up(codes_len, 4) > codes_cap, or >= 2^32 code bits);
 * on an error no code bytes or offsets are written, *d_codes_len is 0 and the
 * header's content is unspecified.
 * d_workspace: 256-byte aligned, mh_encode_workspace_bytes(). The return value
 * covers only argument checks and launch errors. A frame encoded this way goes to
 * mh_build_tables_device (the header) and mh_decode without touching the host.
 * Every call leaves the workspace's symbol histogram zeroed; a caller that
 * zero-filled the workspace once before its first use may pass
 * MH_ENCODE_WORKSPACE_ZEROED in `flags` to skip the per-call clear (one memset
 * launch, ~2 us of a ~33 us frame). */
#define MH_ENCODE_WORKSPACE_ZEROED 0x100u
int mh_encode_frame_device_async(const uint8_t *d_gray, uint32_t width, uint32_t height, uint32_t flags,
                                 uint8_t *d_canon_header, uint8_t *d_codes, uint64_t codes_cap,
                                 uint64_t *d_codes_len, uint32_t *d_block_offsets, uint8_t *d_block_init,
                                 int32_t *d_status, void *d_workspace, size_t workspace_bytes, void *stream);

/* mh_encode_frame_device_async, then one copy and one synchronisation of
 * `stream` to return canon_header and *codes_len on the host; the device status
 * becomes the return value (output byte-identical to mh_encode_frame:
 * HuffmanEncoder.cpp:310-381, HuffmanUtil.cpp:1051-1131, AAPLRenderer.m:374-688). */
int mh_encode_frame_device(const uint8_t *d_gray, uint32_t width, uint32_t height, uint32_t flags,
                           uint8_t canon_header[256], uint8_t *d_codes, uint64_t codes_cap,
                           uint64_t *codes_len, uint32_t *d_block_offsets, uint8_t *d_block_init,
                           void *d_workspace, size_t workspace_bytes, void *stream);

/* Device workspace mh_encode_frames_device_async needs for n_frames frames of
 * width x height. */
size_t mh_encode_frames_workspace_bytes(uint32_t width, uint32_t height, uint32_t n_frames);

/* Batched GPU encode: n_frames independent frames of one size (frame f's pixels at
 * d_gray + f * gray_frame_stride, rows of W bytes), each with its OWN histogram,
 * Huffman tree, canonical header and codes -- byte-identical, frame by frame, to
 * mh_encode_frame (HuffmanEncoder.cpp:310-381, HuffmanUtil.cpp:1051-1131) -- in
 * three launches whatever n_frames (tiled split; one tree workgroup per frame, which
 * also turns the frame's per-tile symbol counts into tile bit offsets; packing), so
 * frames no longer queue behind one workgroup's tree each. Outputs, per frame f:
 * d_canon_headers + 256 f, codes at d_codes + f * codes_frame_stride (16-byte
 * aligned slots; the slot size is the capacity), d_codes_len[f] (optional),
 * d_block_offsets + f * NB, d_block_init + f * NB (optional), d_status[f]
 * (optional; the values of mh_encode_frame_device_async), and d_frame_code_offsets
 * (optional, n_frames + 1 u64 = f * codes_frame_stride): the slots are then one
 * mh_frame batch for mh_decode (all frames must share one canonical table to be
 * decoded in one launch, e.g. block shuffles of one image). A rejected frame writes
 * no codes or offsets and does not affect the others. d_workspace: 256-byte aligned,
 * mh_encode_frames_workspace_bytes(), any content (every part is written before it
 * is read within the call; MH_ENCODE_WORKSPACE_ZEROED is accepted and changes nothing).
 * Asynchronous on `stream`; the return value covers argument checks and launches. */
int mh_encode_frames_device_async(const uint8_t *d_gray, uint64_t gray_frame_stride, uint32_t n_frames,
                                  uint32_t width, uint32_t height, uint32_t flags, uint8_t *d_canon_headers,
                                  uint8_t *d_codes, uint64_t codes_frame_stride, uint64_t *d_codes_len,
                                  uint64_t *d_frame_code_offsets, uint32_t *d_block_offsets, uint8_t *d_block_init,
                                  int32_t *d_status, void *d_workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------- */
/* Streaming from host memory (BASELINE config 5; the reference's per-frame  */
/* command buffer, AAPLRenderer.m:1178-1921).                               */

typedef struct mh_stream mh_stream;

/* A decode stream for frames shaped like `proto` (dims, flags, tables, d_lut;
 * a non-NULL proto->d_block_init means frames carry per-block init bytes; the
 * frame pointers in proto are ignored). It owns n_slots device slots of
 * codes_capacity code bytes each, one HIP stream per slot (its copies, then its
 * decode), and one captured decode graph per slot. Slot i decodes into d_outputs[i] (caller
 * device buffers of round_up(W, 8) * H bytes, 8-byte aligned) or, when
 * d_outputs is NULL, into rasters the stream allocates. */
int mh_stream_create(const mh_frame *proto, uint64_t codes_capacity, uint32_t n_slots,
                     uint8_t *const *d_outputs, mh_stream **out);
/* Queue one frame: H2D copy of its host buffers (pinned memory for a DMA) into
 * the next slot, after that slot's previous decode (same stream), then the slot's
 * decode. codes_bytes includes the MH_CODES_PAD zero bytes; h_block_init must
 * be given iff the stream was created with it. When the host codes follow the
 * block offsets at byte round_up(4*NB, 16) of one buffer, both move in one DMA.
 * Returns the slot in *slot. */
int mh_stream_submit(mh_stream *s, const uint8_t *h_codes, uint64_t codes_bytes,
                     const uint32_t *h_block_offsets, const uint8_t *h_block_init,
                     uint32_t *slot);
/* The slot's output raster (device); valid until n_slots further submits. */
uint8_t *mh_stream_output(mh_stream *s, uint32_t slot, size_t *out_pitch);
/* Each slot copies and decodes on its own hipStream_t (stream order keeps a slot's
 * decode ahead of the copy that reuses it). mh_stream_slot_stream: the stream of
 * `slot`, for events or work that consumes its raster; mh_stream_compute_stream:
 * the stream of the most recent submit. */
void *mh_stream_slot_stream(mh_stream *s, uint32_t slot);
void *mh_stream_compute_stream(mh_stream *s);
int mh_stream_wait(mh_stream *s, uint32_t slot);  /* that slot's decode done */
/* Device-side latency of the slot's most recent frame (waits for it): from the
 * start of its H2D copy to the end of its decode, in milliseconds. */
int mh_stream_slot_time(mh_stream *s, uint32_t slot, float *ms);
int mh_stream_device(mh_stream *s);               /* the HIP device it runs on */
int mh_stream_synchronize(mh_stream *s);
int mh_stream_destroy(mh_stream *s);

/* Stream groups (config 5 on N GPUs of one node): n_members streams, member i on
 * HIP device devices[i] with protos[i] (tables and d_lut resident on that device),
 * n slots each; frames are round-robined over the members in submit order (frame
 * k -> member k mod n). Every call sets the member's device for its duration and
 * restores the caller's. A device may appear more than once. */
typedef struct mh_stream_group mh_stream_group;
int mh_stream_group_create(const mh_frame *protos, uint32_t n_members, const int *devices,
                           uint64_t codes_capacity, uint32_t slots_per_member,
                           mh_stream_group **out);
int mh_stream_group_submit(mh_stream_group *g, const uint8_t *h_codes, uint64_t codes_bytes,
                           const uint32_t *h_block_offsets, const uint8_t *h_block_init,
                           uint32_t *member, uint32_t *slot);
mh_stream *mh_stream_group_member(mh_stream_group *g, uint32_t member);
uint32_t mh_stream_group_size(const mh_stream_group *g);
int mh_stream_group_synchronize(mh_stream_group *g);
int mh_stream_group_destroy(mh_stream_group *g);

/* ---------------------------------------------------------------------- */
/* Host-side producer (CPU, reentrant). Outputs are byte-identical to the   */
/* reference's C++ codec.                                                   */

/* Util.m:233-323 splitIntoBlocksOfSize (zero pad). out: bw*bh*bdim*bdim bytes. */
int mh_split_blocks(const uint8_t *img, uint32_t width, uint32_t height, uint32_t block_dim,
                    uint8_t zero_value, uint8_t *out, size_t out_bytes);

/* Inverse of mh_split_blocks: block order -> W x H raster (crop). */
int mh_merge_blocks(const uint8_t *blocks, uint32_t width, uint32_t height, uint32_t block_dim,
                    uint8_t *out, size_t out_pitch);

/* HuffmanUtil::encodeSignedByteDeltas / decodeSignedByteDeltas
 * (HuffmanUtil.cpp:1133-1145 -> :21-78), applied to n bytes; in == out allowed. */
int mh_encode_signed_byte_deltas(const uint8_t *in, uint8_t *out, size_t n);
int mh_decode_signed_byte_deltas(const uint8_t *in, uint8_t *out, size_t n);

/* Upper bound of the codes bytes mh_encode_huffman / mh_encode_frame write. */
uint64_t mh_codes_bound(uint64_t n_symbols);

/* HuffmanUtil::encodeHuffman (HuffmanUtil.cpp:1051-1131 -> HuffmanEncoder::encode
 * HuffmanEncoder.cpp:310-381): canonical header, MSB-first codes followed by the
 * encoder's 2 zero bytes (*codes_len includes them) and the bit offset of every
 * block_dim*block_dim-th symbol (n_symbols / (block_dim^2) entries). */
int mh_encode_huffman(const uint8_t *symbols, uint64_t n_symbols, uint32_t block_dim,
                      uint8_t canon_header[256], uint8_t *codes, uint64_t codes_cap,
                      uint64_t *codes_len, uint32_t *block_bit_offsets);

/* The renderer's whole producer step (AAPLRenderer.m:374-688) for one 8-bit
 * gray frame: split into zero-padded 8x8 blocks, per-block deltas (unless
 * MH_FLAG_NO_DELTA), encode, block offsets, and MH_CODES_PAD zero bytes of
 * read-ahead after the payload (*codes_len includes them). codes_cap >=
 * mh_codes_bound(NB*64) + 2. block_offsets: NB entries. block_init (optional,
 * NB bytes): when non-NULL, the first delta of every block is moved into it
 * and zeroed (IMPL_DELTAS_AND_INIT_ZERO_DELTA_BEFORE_HUFF_ENCODING,
 * AAPLRenderer.m:449-473). */
int mh_encode_frame(const uint8_t *gray, uint32_t width, uint32_t height, uint32_t flags,
                    uint8_t canon_header[256], uint8_t *codes, uint64_t codes_cap,
                    uint64_t *codes_len, uint32_t *block_offsets, uint8_t *block_init);

/* huff_util.hpp:94-193 huff_generate_canonical_codes: left-justified u16 codes. */
int mh_canonical_codes(const uint8_t canon_header[256], uint16_t codes[256]);

/* HuffmanUtil::parseCanonicalHeader + generateSplitLookupTables(8, 8, ...)
 * (HuffmanUtil.cpp:270-310, :338-667), without module statics. table2 needs
 * room for MH_TABLE2_MAX_ENTRIES entries; *table2_entries = (k+1)*256. */
int mh_build_tables(const uint8_t canon_header[256], mh_lookup_symbol table1[256],
                    mh_lookup_symbol *table2, uint32_t table2_cap, uint32_t *table2_entries);

/* CPU decoders (host, reentrant; never used by the GPU path).
 * HuffmanUtil::decodeHuffmanBits (HuffmanUtil.cpp:673-823; Huffman.h:30): serial
 * decode of n_symbols from the MSB-first stream through the single 65536-entry
 * table (mh_build_single_table); bit_offsets (optional, n_symbols entries) gets
 * each symbol's starting bit. MH_ERR_CAPACITY where the reference asserts
 * (numBytesRead + 2 < huffBuffN). */
int mh_decode_huffman_bits(const mh_lookup_symbol *table, uint64_t n_symbols, const uint8_t *codes,
                           uint64_t codes_bytes, uint8_t *out, uint32_t *bit_offsets);
/* HuffmanUtil::decodeHuffmanBitsFromTables (HuffmanUtil.cpp:830-1046; Huffman.h:42,
 * Huffman.mm:101): the same through the T1/T2 pair (table1_bits = table2_bits = 8,
 * as the reference's tables are built). */
int mh_decode_huffman_bits_from_tables(const mh_lookup_symbol *table1, const mh_lookup_symbol *table2,
                                       uint32_t table2_entries, uint32_t table1_bits, uint32_t table2_bits,
                                       uint64_t n_symbols, const uint8_t *codes, uint64_t codes_bytes,
                                       uint8_t *out, uint32_t *bit_offsets);
/* The CPU twin of mh_decode for one frame: every 8x8 block from its root bit
 * offset with the shader's semantics (AAPLShaders.metal:241-268: 16-bit window,
 * T1/T2, delta fold unless MH_FLAG_NO_DELTA, optional per-block init byte), written
 * into the W x H raster at out_pitch; block rows split over n_threads host threads
 * (0 or 1: the calling thread); each thread decodes eight neighbouring blocks in
 * lock-step. Bytes past codes_bytes read as zero. MH_ERR_CAPACITY if its 128 KB
 * flat table cannot be allocated. */
int mh_decode_frame_cpu(const uint32_t *block_offsets, const uint8_t *codes, uint64_t codes_bytes,
                        const mh_lookup_symbol *table1, const mh_lookup_symbol *table2,
                        uint32_t table2_entries, const uint8_t *block_init, uint32_t width,
                        uint32_t height, uint32_t flags, uint8_t *out, size_t out_pitch,
                        uint32_t n_threads);

/* The 8-byte container header HuffmanEncoder::encode emits ahead of the
 * canonical table (HuffmanEncoder.cpp:326-340: u32 LE 0xFFEEEEDD, u32 LE symbol
 * count) and HuffmanUtil::encodeHuffman drops (HuffmanUtil.cpp:1073-1086). */
#define MH_CONTAINER_HEADER_BYTES 8
#define MH_CONTAINER_MAGIC 0xFFEEEEDDu
int mh_container_header(uint64_t n_symbols, uint8_t header[MH_CONTAINER_HEADER_BYTES]);
/* MH_ERR_INVALID_ARG when the magic word does not match. */
int mh_parse_container_header(const uint8_t header[MH_CONTAINER_HEADER_BYTES], uint64_t *n_symbols);

/* Huffman code lengths (the canonical header) from 256 symbol counts, with the
 * reference tree's tie-breaking (HuffmanEncoder.cpp:29-145). MH_ERR_EMPTY for no
 * symbols, MH_ERR_CODE_TOO_LONG past 16 bits (lengths still written). */
int mh_code_lengths(const uint64_t freq[256], uint8_t canon_header[256]);

/* HuffmanUtil::generateLookupTable (HuffmanUtil.cpp:314-334): 65536 entries. */
int mh_build_single_table(const uint8_t canon_header[256], mh_lookup_symbol table[65536]);

/* ---------------------------------------------------------------------- */
/* Utilities */
const char *mh_error_string(int status);
int mh_device_count(void);
/* sha256 (hex) over the compile flags, sources and headers the library was built
 * from (metalhuffman_amd/build.py). The Python loader refuses a library whose
 * stamp differs from the sources beside it; a debug build's self-check in the
 * spirit of the renderer's DEBUG decode compare (AAPLRenderer.m:616-650). */
const char *mh_build_stamp(void);

#ifdef __cplusplus
}
#endif
#endif /* METALHUFFMAN_H */
