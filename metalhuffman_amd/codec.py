"""Host-side producer API (CPU) -- the reference's `Huffman` facade without module state.

Mirrors the class methods of Shared/Huffman.h:9-77 (ObjC) / HuffmanUtil statics
(Shared/HuffmanUtil.hpp:22-100) with the same names and argument meaning, backed by
the C++ codec in libmetalhuffman_amd.so (csrc/mh_host.cpp). Outputs are
byte-identical to the reference encoder and table builder.

Differences from the reference, by design:
  * no module statics: parseCanonicalHeader returns the canonical codes instead of
    stashing them (HuffmanUtil.cpp:87-102), and generateSplitLookupTables takes the
    canonical header explicitly;
  * errors raise MHError instead of assert() (e.g. a code deeper than 16 bits,
    HuffmanEncoder.cpp:131);
  * the CPU decoders (decodeHuffmanBits*, decode_frame_cpu) are product code in the
    native library (csrc/mh_cpu.cpp, a threaded frame decoder for the reference's CPU
    path); the GPU decoder is the hot path. Neither calls the CPU restatement in
    oracle/, which stays the test-only checker.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional

import numpy as np

from . import _native as N

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def _p(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


BLOCK_DIM = 8


def block_grid(width: int, height: int, block_dim: int = BLOCK_DIM) -> tuple[int, int]:
    """AAPLRenderer.m:753-761: ceil(W/8) x ceil(H/8)."""
    return -(-width // block_dim), -(-height // block_dim)


@dataclasses.dataclass
class EncodedFrame:
    """One frame in the reference's buffer contract (AAPLRenderer.m:374-688)."""
    width: int
    height: int
    canon: np.ndarray           # u8[256] canonical code lengths
    codes: np.ndarray           # u8[payload + MH_CODES_PAD] (huffBuff, read-ahead included)
    block_offsets: np.ndarray   # u32[NB] bit offset of every 8x8 block
    block_init: Optional[np.ndarray] = None  # u8[NB] (INIT_ZERO_DELTA mode) or None
    flags: int = 0

    @property
    def block_width(self) -> int:
        return block_grid(self.width, self.height)[0]

    @property
    def block_height(self) -> int:
        return block_grid(self.width, self.height)[1]

    @property
    def n_blocks(self) -> int:
        return self.block_width * self.block_height

    @property
    def payload_bytes(self) -> int:
        return int(self.codes.size) - N.MH_CODES_PAD

    def tables(self) -> tuple[np.ndarray, np.ndarray]:
        return Huffman.generateSplitLookupTables(self.canon)

    def band(self, by0: int, by1: int) -> "EncodedFrame":
        """Block rows [by0, by1) as a self-contained frame (the
        single-frame split): blocks are independent given their offsets, so a band
        needs only the code bytes from its first block's byte to its last block's
        end. Offsets are rebased to that byte, MH_CODES_PAD zero bytes follow, and
        the height is the band's pixel rows (the last band keeps the frame's partial
        block row). Decoding the band gives rows [8*by0, 8*by0 + height) of the frame."""
        bw, bh = self.block_width, self.block_height
        if not 0 <= by0 < by1 <= bh:
            raise ValueError(f"block rows [{by0}, {by1}) outside [0, {bh})")
        b0, b1 = by0 * bw, by1 * bw
        offs = self.block_offsets
        base = int(offs[b0]) >> 3
        end_bits = int(offs[b1]) if b1 < self.n_blocks else 8 * self.payload_bytes
        end = (end_bits + 7) >> 3
        codes = np.zeros(end - base + N.MH_CODES_PAD, np.uint8)
        codes[: end - base] = self.codes[base:end]
        band_offs = (offs[b0:b1].astype(np.int64) - 8 * base).astype(np.uint32)
        init = None if self.block_init is None else self.block_init[b0:b1].copy()
        height = min(self.height, 8 * by1) - 8 * by0
        return EncodedFrame(self.width, height, self.canon, codes, band_offs, init, self.flags)


class Huffman:
    """Stateless mirror of the reference's `Huffman` class (Shared/Huffman.h)."""

    # +parseCanonicalHeader: (Huffman.h:14, HuffmanUtil.cpp:270-310)
    @staticmethod
    def parseCanonicalHeader(canonData) -> np.ndarray:
        canon = _u8(canonData)
        if canon.size != 256:
            raise ValueError("canonical header must be 256 bytes")
        codes = np.zeros(256, np.uint16)
        N.check(N.lib().mh_canonical_codes(_p(canon), _p(codes, _u16p)), "parseCanonicalHeader")
        return codes

    # +generateLookupTable:lookupTableNumEntries: (Huffman.h:18, HuffmanUtil.cpp:314-334)
    @staticmethod
    def generateLookupTable(canonData) -> np.ndarray:
        canon = _u8(canonData)
        table = np.zeros(65536 * 2, np.uint8)
        N.check(N.lib().mh_build_single_table(_p(canon), _p(table)), "generateLookupTable")
        return table

    # +generateSplitLookupTables:table2NumBits:table1:table2: (Huffman.h:21-24,
    # HuffmanUtil.cpp:338-667). Returns (T1, T2) as raw 2-byte-entry arrays.
    @staticmethod
    def generateSplitLookupTables(canonData, table1NumBits: int = 8, table2NumBits: int = 8):
        if (table1NumBits, table2NumBits) != (8, 8):
            # the reference's table sizes are the compile-time HUFF_TABLE{1,2}_SIZE
            # (AAPLShaderTypes.h:120-123); only the 8/8 split is a valid contract
            raise ValueError("only the 8+8 split (HUFF_TABLE1/2_NUM_BITS) is supported")
        canon = _u8(canonData)
        t1 = np.zeros(512, np.uint8)
        t2 = np.zeros(N.MH_TABLE2_MAX_ENTRIES * 2, np.uint8)
        ent = ctypes.c_uint32(0)
        N.check(N.lib().mh_build_tables(_p(canon), _p(t1), _p(t2), N.MH_TABLE2_MAX_ENTRIES,
                                        ctypes.byref(ent)), "generateSplitLookupTables")
        return t1, t2[: 2 * ent.value].copy()

    # +encodeHuffman:inNumBytes:outFileHeader:outCanonHeader:outHuffCodes:
    #  outBlockBitOffsets:width:height:blockDim: (Huffman.h:62-70, HuffmanUtil.cpp:1051-1131)
    @staticmethod
    def encodeHuffman(inBytes, width: int, height: int, blockDim: int = BLOCK_DIM):
        """-> (fileHeader, canonHeader, huffCodes, blockBitOffsets).

        fileHeader is empty, as in the reference (HuffmanUtil.cpp:1073-1086 never
        copies the encoder's header bytes out); huffCodes carries the encoder's
        2 zero bytes of read-ahead."""
        sym = _u8(inBytes)
        if sym.size == 0:
            raise N.MHError(-8, "encodeHuffman")
        cap = int(N.lib().mh_codes_bound(sym.size))
        canon = np.zeros(256, np.uint8)
        codes = np.zeros(cap, np.uint8)
        stride = blockDim * blockDim
        offs = np.zeros(max(1, sym.size // stride), np.uint32)
        ln = ctypes.c_uint64(0)
        N.check(N.lib().mh_encode_huffman(_p(sym), sym.size, blockDim, _p(canon), _p(codes), cap,
                                          ctypes.byref(ln), _p(offs, _u32p)), "encodeHuffman")
        return (np.zeros(0, np.uint8), canon, codes[: ln.value].copy(),
                offs[: sym.size // stride].copy())

    # +decodeHuffmanBits:numSymbolsToDecode:huffBuff:huffBuffN:outBuffer:bitOffsetTable:
    # (Huffman.h:30-35, HuffmanUtil.cpp:673-823). -> (symbols, bitOffsetTable)
    @staticmethod
    def decodeHuffmanBits(huffSymbolTable, numSymbolsToDecode: int, huffBuff, bitOffsets: bool = False):
        table = _u8(huffSymbolTable)
        if table.size != 65536 * 2:
            raise ValueError("the single lookup table has 65536 two-byte entries")
        buf = _u8(huffBuff)
        out = np.zeros(int(numSymbolsToDecode), np.uint8)
        offs = np.zeros(int(numSymbolsToDecode), np.uint32) if bitOffsets else None
        N.check(N.lib().mh_decode_huffman_bits(_p(table), out.size, _p(buf), buf.size, _p(out),
                                               _p(offs, _u32p) if offs is not None else None),
                "decodeHuffmanBits")
        return out, offs

    # +decodeHuffmanBitsFromTables:huffSymbolTable2:table1BitNum:table2BitNum:
    #  numSymbolsToDecode:huffBuff:huffBuffN:outBuffer:bitOffsetTable: (Huffman.h:42-50,
    # Huffman.mm:101, HuffmanUtil.cpp:830-1046). -> (symbols, bitOffsetTable)
    @staticmethod
    def decodeHuffmanBitsFromTables(huffSymbolTable1, huffSymbolTable2, table1BitNum: int,
                                    table2BitNum: int, numSymbolsToDecode: int, huffBuff,
                                    bitOffsets: bool = False):
        t1, t2, buf = _u8(huffSymbolTable1), _u8(huffSymbolTable2), _u8(huffBuff)
        if t1.size != 512:
            raise ValueError("T1 has 256 two-byte entries")
        out = np.zeros(int(numSymbolsToDecode), np.uint8)
        offs = np.zeros(int(numSymbolsToDecode), np.uint32) if bitOffsets else None
        N.check(N.lib().mh_decode_huffman_bits_from_tables(
            _p(t1), _p(t2), t2.size // 2, int(table1BitNum), int(table2BitNum), out.size, _p(buf), buf.size,
            _p(out), _p(offs, _u32p) if offs is not None else None), "decodeHuffmanBitsFromTables")
        return out, offs

    @staticmethod
    def containerHeader(n_symbols: int) -> np.ndarray:
        """The 8-byte header HuffmanEncoder::encode emits (HuffmanEncoder.cpp:326-340)
        and encodeHuffman drops: u32 LE 0xFFEEEEDD, u32 LE symbol count."""
        out = np.zeros(8, np.uint8)
        N.check(N.lib().mh_container_header(int(n_symbols), _p(out)), "containerHeader")
        return out

    @staticmethod
    def parseContainerHeader(header) -> int:
        """Symbol count of a container header (MHError on a wrong magic word)."""
        h = _u8(header)
        if h.size != 8:
            raise N.MHError(-1, "parseContainerHeader")
        n = ctypes.c_uint64(0)
        N.check(N.lib().mh_parse_container_header(_p(h), ctypes.byref(n)), "parseContainerHeader")
        return int(n.value)

    # +encodeSignedByteDeltas: / +decodeSignedByteDeltas: (Huffman.h:72-76)
    @staticmethod
    def encodeSignedByteDeltas(data) -> np.ndarray:
        a = _u8(data)
        out = np.empty_like(a)
        N.check(N.lib().mh_encode_signed_byte_deltas(_p(a), _p(out), a.size), "encodeSignedByteDeltas")
        return out

    @staticmethod
    def decodeSignedByteDeltas(deltas) -> np.ndarray:
        a = _u8(deltas)
        out = np.empty_like(a)
        N.check(N.lib().mh_decode_signed_byte_deltas(_p(a), _p(out), a.size), "decodeSignedByteDeltas")
        return out

    # snake_case aliases
    parse_canonical_header = parseCanonicalHeader
    generate_lookup_table = generateLookupTable
    generate_split_lookup_tables = generateSplitLookupTables
    encode_huffman = encodeHuffman
    decode_huffman_bits = decodeHuffmanBits
    decode_huffman_bits_from_tables = decodeHuffmanBitsFromTables
    encode_signed_byte_deltas = encodeSignedByteDeltas
    decode_signed_byte_deltas = decodeSignedByteDeltas


def split_blocks(img: np.ndarray, block_dim: int = BLOCK_DIM, zero_value: int = 0) -> np.ndarray:
    """Util.m:233-323 splitIntoBlocksOfSize (zero padded) -> block-order bytes."""
    img = _u8(img)
    h, w = img.shape
    bw, bh = block_grid(w, h, block_dim)
    out = np.empty(bw * bh * block_dim * block_dim, np.uint8)
    N.check(N.lib().mh_split_blocks(_p(img), w, h, block_dim, zero_value, _p(out), out.size),
            "split_blocks")
    return out


def merge_blocks(blocks: np.ndarray, width: int, height: int, block_dim: int = BLOCK_DIM) -> np.ndarray:
    blocks = _u8(blocks)
    out = np.empty((height, width), np.uint8)
    N.check(N.lib().mh_merge_blocks(_p(blocks), width, height, block_dim, _p(out), width),
            "merge_blocks")
    return out


def encode_frame(gray: np.ndarray, flags: int = 0, init_zero_delta: bool = False) -> EncodedFrame:
    """The renderer's producer step (AAPLRenderer.m:374-688) for one 8-bit frame."""
    gray = _u8(gray)
    if gray.ndim != 2:
        raise ValueError("expected a 2-D uint8 image")
    h, w = gray.shape
    bw, bh = block_grid(w, h)
    nb = bw * bh
    cap = int(N.lib().mh_codes_bound(nb * 64)) + 2
    canon = np.zeros(256, np.uint8)
    codes = np.zeros(cap, np.uint8)
    offs = np.zeros(nb, np.uint32)
    init = np.zeros(nb, np.uint8) if init_zero_delta else None
    ln = ctypes.c_uint64(0)
    N.check(N.lib().mh_encode_frame(_p(gray), w, h, flags, _p(canon), _p(codes), cap, ctypes.byref(ln),
                                    _p(offs, _u32p), _p(init) if init is not None else None),
            "encode_frame")
    return EncodedFrame(w, h, canon, codes[: ln.value].copy(), offs, init, flags)


def decode_frame_cpu(ef: EncodedFrame, threads: int = 1) -> np.ndarray:
    """CPU twin of the GPU decode for one frame (mh_decode_frame_cpu): the shader
    semantics per block, straight to the H x W raster, on `threads` host threads."""
    t1, t2 = ef.tables()
    out = np.zeros((ef.height, ef.width), np.uint8)
    offs = np.ascontiguousarray(ef.block_offsets, np.uint32)
    init = np.ascontiguousarray(ef.block_init, np.uint8) if ef.block_init is not None else None
    N.check(N.lib().mh_decode_frame_cpu(_p(offs, _u32p), _p(ef.codes), ef.codes.size, _p(t1), _p(t2),
                                        t2.size // 2, _p(init) if init is not None else None, ef.width,
                                        ef.height, ef.flags, _p(out), ef.width, int(threads)),
            "mh_decode_frame_cpu")
    return out
