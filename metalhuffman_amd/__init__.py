"""metalhuffman_amd -- MI355X-native Huffman block decoder (drop-in for the decode path
of mdejong/MetalHuffman).

  * include/metalhuffman.h          C-ABI (the drop-in boundary)
  * csrc/mh_decode.hip              hand-written gfx950 decode kernel
  * csrc/mh_host.cpp                host producer: encoder, canonical codes, T1/T2
  * csrc/mh_cpu.cpp                 the reference's CPU decoders + a threaded CPU frame decoder
  * codec.Huffman                   the reference's `Huffman` facade (Shared/Huffman.h)
  * decoder.decode / DeviceFrames   GPU decode of one frame or a batch
  * decoder.DeviceTables            T1/T2 + prepared table (uploaded, or built on the device)
  * encoder.Encoder                 GPU encoder (encode / encode_async: no host sync)
  * stream                          streaming from host memory (config 5)
  * dist                            frame sharding, single-frame bands, table broadcast
"""
from ._native import EXPORTS, LIB_PATH, MH_CODES_PAD, MH_FLAG_LANE_PAIRS, MH_FLAG_NO_DELTA, MHError, lib
from .codec import (BLOCK_DIM, EncodedFrame, Huffman, block_grid, decode_frame_cpu, encode_frame, merge_blocks,
                    split_blocks)

__all__ = [
    "EXPORTS", "LIB_PATH", "MH_CODES_PAD", "MH_FLAG_LANE_PAIRS", "MH_FLAG_NO_DELTA", "MHError", "lib", "BLOCK_DIM",
    "EncodedFrame", "Huffman", "block_grid", "decode_frame_cpu", "encode_frame", "merge_blocks", "split_blocks",
]
__version__ = "0.1.0"
