/*
 * mh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of mdejong/MetalHuffman's Huffman block codec, used
 * as the CPU checker for the MI355X decoder. Only tests/, the smoke() entry
 * in __graft_entry__.py and the cpu_baseline leg of bench.py may load this
 * library; the product (metalhuffman_amd/) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference root, Shared/...). Parity pinning: see oracle/README.md --
 * the encoder half is checked byte-for-byte against the real reference
 * encoder (Shared/HuffmanEncoder.cpp compiled unmodified into oracle/_ref),
 * the table builder / decoders against the SHA-256 golden vectors recorded in
 * SURVEY.md 8(c) and the TEST_6x4_NOT_SQUARE known-answer arrays
 * (Shared/HuffRenderFrame.m:250-300).
 */
#ifndef MH_ORACLE_H
#define MH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Shared/HuffmanLookupSymbol.h:7-10 -- 2-byte table entry. */
typedef struct {
  uint8_t symbol;
  uint8_t bitWidth;
} orc_sym;

#define ORC_OK 0
#define ORC_ERR_ARG (-1)
#define ORC_ERR_TOO_LONG (-2) /* Huffman depth > 16: reference asserts (HuffmanEncoder.cpp:131) */
#define ORC_ERR_CAP (-3)
#define ORC_ERR_EMPTY (-4)

/* Util.m:233-323 -- zero-padded split of a W x H byte image into bdim x bdim
 * blocks, block order by*bw+bx, row-major inside a block. */
int orc_split_blocks(const uint8_t *img, uint32_t w, uint32_t h, uint32_t bdim,
                     uint32_t bw, uint32_t bh, uint8_t zero, uint8_t *out);

/* HuffmanUtil.cpp:21-47 (encodeDelta) / :49-78 (decodePlusDelta), int8 wrap,
 * applied in place to n bytes. */
void orc_delta_encode(uint8_t *buf, size_t n);
void orc_delta_decode(uint8_t *buf, size_t n);

/* HuffmanEncoder.cpp:29-145 (frequency, node array, tree, code depth) +
 * huff_util.hpp:45-68 -> 256-byte canonical header of code lengths. */
int orc_code_lengths(const uint8_t *in, uint32_t n, uint8_t canon[256]);

/* huff_util.hpp:94-193 -- canonical, left-justified 16-bit codes. */
void orc_canonical_codes(const uint8_t canon[256], uint16_t codes[256]);

/* HuffmanEncoder.cpp:310-381 + HuffmanUtil.cpp:1051-1131 -- full encode:
 * canonical header, MSB-first codes + 2 zero bytes, and the bit offset of
 * every `stride`-th symbol (stride = blockDim*blockDim) in offsets[]. */
int orc_huffman_encode(const uint8_t *in, uint32_t n, uint32_t stride,
                       uint8_t canon[256], uint8_t *codes, uint64_t codes_cap,
                       uint64_t *codes_len, uint32_t *offsets);

/* HuffmanUtil.cpp:338-667 -- 8+8 split tables. t2 needs room for
 * 257*256 entries; *t2_entries receives (k+1)*256. */
int orc_split_tables(const uint8_t canon[256], orc_sym t1[256], orc_sym *t2,
                     uint32_t t2_cap, uint32_t *t2_entries);

/* HuffmanUtil.cpp:314-334 -- single 65536-entry table. */
int orc_single_table(const uint8_t canon[256], orc_sym t[65536]);

/* HuffmanUtil.cpp:830-1046 -- serial whole-stream decode from T1/T2.
 * bit_offsets may be NULL. */
void orc_decode_from_tables(const orc_sym *t1, const orc_sym *t2, uint32_t nsym,
                            const uint8_t *buf, uint8_t *out, uint32_t *bit_offsets);

/* HuffmanUtil.cpp:673-823 -- serial decode from the single 64K table. */
void orc_decode_single_table(const orc_sym *t, uint32_t nsym, const uint8_t *buf,
                             uint8_t *out, uint32_t *bit_offsets);

/* AAPLShaders.metal:127-178 (huffDecodeSymbol), :241-268 (decode step + delta),
 * :291-445 (64 steps per block over the W12x4 + W16 passes), :449-518
 * (block -> raster reorder + crop). Writes a W x H raster at out (pitch W).
 * block_init may be NULL (prev starts at 0). delta=0 emits raw symbols
 * (IMPL_DELTAS_BEFORE_HUFF_ENCODING off, AAPLShaders.metal:263-265). */
int orc_decode_frame_shader(const uint32_t *block_offsets, const uint8_t *codes,
                            const orc_sym *t1, const orc_sym *t2, uint32_t w,
                            uint32_t h, uint32_t bw, uint32_t bh,
                            const uint8_t *block_init, int delta, uint8_t *out);

/* The whole producer pipeline of AAPLRenderer.m:374-688 for 8x8 blocks with
 * deltas on: split -> per-block delta -> encode -> offsets per block. codes
 * receives the encoder's bytes followed by 2 more zero bytes (the renderer's
 * read-ahead, AAPLRenderer.m:576-585), *codes_len counts all of them. */
int orc_encode_frame(const uint8_t *img, uint32_t w, uint32_t h, uint8_t canon[256],
                     uint8_t *codes, uint64_t codes_cap, uint64_t *codes_len,
                     uint32_t *block_offsets);

/* CPU baseline: decode n_frames block-order streams with
 * orc_decode_from_tables on n_threads threads (frame-parallel), repeating the
 * whole set `reps` times. Returns wall seconds. */
double orc_time_decode_frames(const orc_sym *t1, const orc_sym *t2, uint32_t nsym,
                              const uint8_t *const *bufs, uint8_t *const *outs,
                              uint32_t n_frames, uint32_t n_threads, uint32_t reps);

/* CPU baseline, full pipeline: as orc_time_decode_frames, then each frame's
 * block-order deltas are integrated per block and merged into its W x H raster
 * (decode + undelta + raster, what a CPU consumer of the reference's buffers does). */
double orc_time_decode_pipeline(const orc_sym *t1, const orc_sym *t2, uint32_t w, uint32_t h,
                                const uint8_t *const *bufs, uint8_t *const *rasters,
                                uint32_t n_frames, uint32_t n_threads, uint32_t reps);

#ifdef __cplusplus
}
#endif
#endif /* MH_ORACLE_H */
