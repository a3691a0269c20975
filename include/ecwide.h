/*
 * ecwide.h — C ABI of the MI355X wide-stripe erasure-coding engine.
 *
 * This is the drop-in boundary for ECWide-C's codec (`libcodec.so`,
 * loaded by NativeCodec.java:213-215). Every entry point is plain C: raw
 * pointers, sizes and int status codes; no torch or HIP types appear in a
 * signature (streams are passed as `void*` = hipStream_t, NULL = default).
 *
 * Reference interface each function replaces (paths relative to the
 * reference repository root):
 *
 *   ecw_scheme_from_ini       CodingScheme.getFromConfig   ECWide-C/src/CodingScheme.java:66-113
 *   ecw_scheme_init           CodingScheme ctors           ECWide-C/src/CodingScheme.java:22-48
 *   ecw_codec_create          NativeCodec ctors (R,T,L,C)  ECWide-C/src/NativeCodec.java:20-109
 *                             + generateEncodeMatrix       ECWide-C/src/native/NativeCodec.cc:12-64
 *                             + initEncodeTable            ECWide-C/src/native/NativeCodec.cc:66-88
 *                             + initDecodeTable            ECWide-C/src/native/NativeCodec.cc:90-111
 *                             + initPartialDecodeTable     ECWide-C/src/native/NativeCodec.cc:113-135
 *   ecw_codec_encode_matrix   NativeCodec.getEncodeMatrix  ECWide-C/src/NativeCodec.java:127-131
 *   ecw_codec_encode_gftbl    NativeCodec.getEncodeGftbl   ECWide-C/src/NativeCodec.java:133-137
 *   ecw_codec_decode_gftbl    NativeCodec.getDecodeGftbl   ECWide-C/src/NativeCodec.java:139-143
 *   ecw_encode                encodeData                   ECWide-C/src/native/NativeCodec.cc:137-219
 *   ecw_decode                decodeData                   ECWide-C/src/native/NativeCodec.cc:221-249
 *   ecw_partial_decode        partialDecodeData            ECWide-C/src/native/NativeCodec.cc:251-282
 *   ecw_xor_intermediate      xorIntemediate               ECWide-C/src/native/NativeCodec.cc:284-323
 *   ecw_*_dev                 the same operations on HBM-resident blocks (stream-ordered)
 *   ecw_encode_batch_dev /    batches of independent stripes in one launch (north_star:
 *   ecw_repair_batch_dev      "stripes are independent by byte range")
 *   ecw_repair / ecw_repair_sources
 *                             the flat fan-in of a CL single-block repair,
 *                             ClMetadataManager.getChunkRepairTask  ECWide-C/src/ClMetadataManager.java:137-257
 *
 * Conventions (mirroring the reference):
 *   - the caller owns every buffer; the library borrows pointers for the call;
 *   - data arrives as arrays of per-block pointers (`const uint8_t* const*`);
 *   - output order of encode is [G_0..G_{m-1}, L_0..L_{g-1}] (BufferUnit.java:60-68);
 *   - unlike the reference (all void, nothing validated) every call validates
 *     and returns an ecw_status; nothing calls exit();
 *   - no static mutable state: all tables live in the codec; a codec may be
 *     used from several host threads as long as each call uses its own
 *     stream (host-pointer calls serialise on an internal per-codec lock).
 */
#ifndef ECWIDE_H_
#define ECWIDE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECW_ABI_VERSION 1

typedef enum ecw_status {
  ECW_OK = 0,
  ECW_EINVAL = -1,       /* bad argument (null pointer, bad size, k+m > 256 ...) */
  ECW_ENOMEM = -2,       /* host or device allocation failed */
  ECW_EDEVICE = -3,      /* a HIP runtime call failed (no GPU, launch failure ...) */
  ECW_EALIGN = -4,       /* device pointer / stride not 16-byte aligned */
  ECW_EUNSUPPORTED = -5, /* operation the reference does not support either */
  ECW_EPARSE = -6,       /* malformed scheme.ini */
  ECW_EIO = -7           /* file could not be read */
} ecw_status;

/* Code types, same letters as NativeCodec.codeType (NativeCodec.java:9). */
#define ECW_CODE_RS 'R'
#define ECW_CODE_TL 'T'
#define ECW_CODE_LRC 'L'
#define ECW_CODE_CL 'C'

/* Local-parity semantics of encode.
 *  ECW_LOCAL_XOR     — L_t = XOR of group t's data blocks: the combined-locality
 *                      code as designed (paper p.238), equal to ECWide-H
 *                      l_encode (ECWide-H/proxy/encode.cpp:113-143) and to
 *                      what decodeData assumes when it XORs a group back.
 *  ECW_LOCAL_LITERAL — bit-exact with ECWide-C encodeData: its XOR table is
 *                      built from an all-zero matrix (NativeCodec.cc:181-186),
 *                      so every L block comes out 0x00.
 * Global parities are identical in both modes. */
#define ECW_LOCAL_XOR 0
#define ECW_LOCAL_LITERAL 1

/* xorIntemediate semantics.
 *  ECW_XORI_XOR     — target[i] ^= source[i] on every call (the intent).
 *  ECW_XORI_LITERAL — the reference's static `flag` is tested the wrong way
 *                     round (NativeCodec.cc:287-292): the first call on a
 *                     codec writes zeros into target, later calls XOR. */
#define ECW_XORI_XOR 0
#define ECW_XORI_LITERAL 1

/* Scheme geometry (CodingScheme fields, CodingScheme.java:8-19). */
typedef struct ecw_scheme {
  char code_type;          /* 'R', 'T', 'L' or 'C' */
  int k;                   /* data blocks */
  int global_parity_num;   /* m (globalParityNum) */
  int group_data_num;      /* r (groupDataNum), -1 for RS/TL */
  int group_num;           /* ceil(k/r) for LRC/CL, 0 otherwise */
  int rack_nodes_num;      /* m+1 (CL), m (TL), -1 (LRC), 0 (RS) */
  int rack_num;            /* see CodingScheme ctors; -1 for LRC, 0 for RS */
  int chunk_size_bits;     /* log2(chunk size) when parsed from ini, else -1 */
  size_t chunk_size;       /* B, bytes per block */
} ecw_scheme;

/* Codec-derived counts (NativeCodec fields, NativeCodec.java:4-18). */
typedef struct ecw_codec_info {
  char code_type;
  int node_index;
  int multinode;
  int local_mode;
  int encode_data_num;     /* encodeDataNum */
  int decode_data_num;     /* decodeDataNum */
  int partial_decode_num;  /* partialDecodeNum (0 for RS/LRC) */
  int global_num;          /* globalNum = m */
  int group_num;           /* groupNum */
  int group_data_num;      /* groupDataNum */
  int rack_per_group;      /* rackPerGroup (CL only) */
  int parity_num;          /* outputs of encode: m (+ groupNum for L/C) */
  size_t chunk_size;
} ecw_codec_info;

typedef struct ecw_codec ecw_codec;

/* ---- library ---------------------------------------------------------- */
int ecw_abi_version(void);
const char* ecw_status_string(int status);
/* Number of visible HIP devices (0 on a host without GPU, never an error). */
int ecw_device_count(void);

/* ---- scheme ----------------------------------------------------------- */
/* Build a scheme exactly as the CodingScheme constructors do. For RS/TL
 * `group_data_num` is ignored. */
int ecw_scheme_init(ecw_scheme* out, char code_type, int k, int m, int group_data_num,
                    size_t chunk_size);
/* Parse `codeType`, `k`, `groupDataNum`, `globalParityNum`, `chunkSizeBits`
 * from a scheme.ini file (ECWide-C/config/scheme.ini), as
 * CodingScheme.getFromConfig does. */
int ecw_scheme_from_ini(const char* path, ecw_scheme* out);
/* Same, from the file's text. */
int ecw_scheme_from_ini_text(const char* text, ecw_scheme* out);

/* ---- codec ------------------------------------------------------------ */
/* Create a codec for `scheme` as seen from 1-based `node_index`.
 * `multinode` selects the multi-node partial encode (ECTaskProcessor.java:
 * 267-291): node i holds data group g-i, encode writes the m partial global
 * parities over that group's columns of the stripe's Cauchy matrix plus the
 * group's local parity (m+1 outputs); XOR-merging the partials of all nodes
 * (xorIntemediate) gives the single-node global parities. The reference's
 * own column slice is misaligned (NativeCodec.cc:46-58), so this mode
 * implements the intended columns.
 * `device` is the HIP device ordinal used for every device-side call;
 * no device work happens until the first encode/decode call, so a codec can
 * be created (and its matrices inspected) on a host without a GPU. */
int ecw_codec_create(const ecw_scheme* scheme, int node_index, int multinode, int local_mode,
                     int device, ecw_codec** out);
void ecw_codec_destroy(ecw_codec* codec);
/* A codec for an arbitrary rows x k GF(2^8) coefficient matrix (row-major),
 * no local groups: encode computes parity[l] = sum_j matrix[l][j] * data[j],
 * exactly ISA-L's ec_encode_data with ec_init_tables(k, rows, matrix)
 * (isal:erasure_code/ec_highlevel_func.c:33-43; ECWide-H/proxy/encode.cpp:
 * 129-130, 161-162, 187-188, 222-223 are such calls). code_type 'M'. */
int ecw_matrix_codec_create(const uint8_t* matrix, int k, int rows, int device, ecw_codec** out);
int ecw_codec_get_info(const ecw_codec* codec, ecw_codec_info* out);
int ecw_codec_set_xori_mode(ecw_codec* codec, int xori_mode);
/* Copy out the m x k encode matrix (row-major), the 32*k*m ISA-L layout
 * gf tables, and the 32*ddn / 32*pdn decode tables. `len` must equal the
 * size the reference allocates (NativeCodec.java:101-104). */
int ecw_codec_encode_matrix(const ecw_codec* codec, uint8_t* out, size_t len);
int ecw_codec_encode_gftbl(const ecw_codec* codec, uint8_t* out, size_t len);
int ecw_codec_decode_gftbl(const ecw_codec* codec, uint8_t* out, size_t len);
int ecw_codec_partial_decode_gftbl(const ecw_codec* codec, uint8_t* out, size_t len);

/* ---- host-memory entry points (blocking; mirror the JNI natives) -------
 * `len` is the number of bytes per block (the reference always passes
 * chunkSize; any len >= 0 is accepted). Each copies the inputs into HBM,
 * runs the HIP kernels and copies the outputs back. */
int ecw_encode(ecw_codec* codec, const uint8_t* const* data, uint8_t* const* parity, size_t len);
int ecw_decode(ecw_codec* codec, const uint8_t* const* data, uint8_t* target, size_t len);
int ecw_partial_decode(ecw_codec* codec, const uint8_t* const* data, uint8_t* target,
                       size_t len);
int ecw_xor_intermediate(ecw_codec* codec, const uint8_t* const* source, uint8_t* const* target,
                         size_t len);

/* Encode `stripes` independent stripes held in host memory in one call:
 * data[s*k + j], parity[s*parity_num + i]. Small blocks (ECWide-H's 4 KiB
 * chunks) are packed into one HBM slab per batch, so a batch costs one
 * launch instead of one per stripe. */
int ecw_encode_stripes(ecw_codec* codec, int stripes, const uint8_t* const* data, uint8_t* const* parity,
                       size_t len);

/* Flat CL single-block repair on host memory: `blocks` holds every block of
 * one stripe in slab order [D.., G.., L..] (the lost one may be NULL);
 * `out` receives the rebuilt `lost_block` (D or L). */
int ecw_repair(ecw_codec* codec, const uint8_t* const* blocks, int lost_block, uint8_t* out, size_t len);

/* NUMA-local pinned host staging for the host-memory entry points. The
 * reference's blocks are host buffers (Java direct ByteBuffers filled from
 * files, BufferUnit.java:53-68, FileOp.java:7-21); the host-memory calls move
 * them over PCIe, at DMA rate only from pinned memory, and across the
 * inter-socket fabric when the buffer sits on the other socket's DRAM.
 * ecw_host_alloc maps `bytes` (rounded up to 4 KiB) of zeroed host memory
 * with its pages preferred on the NUMA node of `device`'s PCIe root (sysfs),
 * faults them in and registers them with the GPU runtime (pinned).
 * *numa_node (optional) receives the node the pages were found on (sampled;
 * -1 when unknown or spread). Free with ecw_host_free. No reference
 * counterpart (placement of the caller's buffers). ECW_EDEVICE without a GPU. */
int ecw_host_alloc(int device, size_t bytes, void** out, int* numa_node);
/* The same with the pages preferred on NUMA node `node` (-1: `device`'s node),
 * registered for `device`: staging next to another socket's DRAM, e.g. where
 * the files' page cache lives, or a local-versus-remote A/B. */
int ecw_host_alloc_node(int device, int node, size_t bytes, void** out, int* numa_node);
int ecw_host_free(void* ptr);
/* NUMA node of `device` (-1 when unknown or no such device). */
int ecw_device_numa_node(int device);

/* Counters of the resident small-request service on `device` (host-memory
 * calls of blocks up to 64 KiB: ecw_encode of one stripe, and the XORs of
 * ecw_decode / ecw_partial_decode / ecw_repair / ecw_xor_intermediate), for
 * callers that mix small and bulk calls (ECWide-H's proxy threads,
 * ECWide-H/proxy/proxy.cpp:2001-2012) to see the service's hit rate:
 * out[0] requests served, out[1] eligible requests that took the launch path
 * instead (bulk work held the service off, or it was stopping), out[2]
 * epochs launched, out[3] 1 if the service has turned itself off after a HIP
 * error. No reference counterpart (observability). ECW_OK; zeros for a
 * device the service never ran on. */
int ecw_service_counters(int device, unsigned long long out[4]);

/* ---- launch schedule (tuning; no reference counterpart) ----------------
 * Process-wide knobs of HOW the kernels are launched: the tile order and the
 * write windows. None changes a result byte (tested against
 * the oracle at every setting), only the order and timing of HBM accesses.
 * A field of -1 leaves that choice to the library (the default everywhere:
 * the per-layout choice DESIGN.md §4 measures). The environment variables
 * ECW_XOR_SCHED="K,ORDER[,LOG2P,W]", ECW_WRITE_WINDOW=off|on|"LOG2P,W" and
 * ECW_XCD_REMAP=0|1 seed the schedule once, at the first launch or schedule
 * call; after that only ecw_set_schedule changes it (the environment is never
 * read per launch). Every launch takes one consistent copy, so the schedule
 * may be set from any thread; launches already queued keep theirs. */
typedef struct ecw_schedule {
  int xor_skew;         /* XOR reduce: column tiles per workgroup, read diagonally: 1, 2 or 4 */
  int xor_order;        /* XOR reduce: 0 = groups stripe-major, 1 = column-major */
  int xor_window_log2p; /* XOR reduce write window: period of 2^log2p ticks of the 100 MHz clock, 4..24 */
  int xor_window_width; /*   stores wait for the first `width` ticks of every period; 0 = no window */
  int enc_window_log2p; /* encode write window: period, 4..24 */
  int enc_window_width; /*   width in ticks; 0 = no window */
  int xcd_remap;        /* per-XCD contiguous tile order of the encode and the XOR: 0 or 1 */
} ecw_schedule;
/* Set the schedule (NULL: every field back to -1). A window with only one of
 * log2p / width set takes the default for the other (2^11 ticks, 64).
 * ECW_EINVAL, and nothing changed, for a value out of range or a skew the
 * library was not built with. */
int ecw_set_schedule(const ecw_schedule* schedule);
int ecw_get_schedule(ecw_schedule* out);

/* ---- device-memory entry points (asynchronous on `stream`) -------------
 * All pointers are HBM addresses, 16-byte aligned. The pointer arrays
 * themselves are host arrays (copied into the kernel arguments). */
int ecw_encode_dev(ecw_codec* codec, const uint8_t* const* d_data, uint8_t* const* d_parity,
                   size_t len, void* stream);
int ecw_decode_dev(ecw_codec* codec, const uint8_t* const* d_data, uint8_t* d_target,
                   size_t len, void* stream);
int ecw_partial_decode_dev(ecw_codec* codec, const uint8_t* const* d_data, uint8_t* d_target,
                           size_t len, void* stream);
int ecw_xor_intermediate_dev(ecw_codec* codec, const uint8_t* const* d_source,
                             uint8_t* const* d_target, size_t len, void* stream);
/* Encode `stripes` stripes of separately placed HBM blocks in ONE launch (the
 * reference's per-block pointer convention, NativeCodec.cc:158-166, batched):
 * d_data_ptrs and d_parity_ptrs are DEVICE arrays (8-byte aligned) of
 * stripes*k data block pointers (stripe-major) and stripes*parity_num output
 * pointers ([G_0..G_{m-1}, L_0..L_{g-1}] per stripe). Every block is `len`
 * bytes, 16-byte aligned (the caller's guarantee: the pointers are not read
 * on the host). Codecs with local groups but no global row (m = 0) are
 * ECW_EUNSUPPORTED here. */
int ecw_encode_ptrs_dev(ecw_codec* codec, int stripes, const uint8_t* const* d_data_ptrs,
                        uint8_t* const* d_parity_ptrs, size_t len, void* stream);
/* dst[s] = XOR of src[s*n + 0 .. s*n + n-1] for every stripe s, one launch: the
 * decode / partial decode / CL repair of a batch of stripes whose blocks are
 * separately placed (d_src_ptrs, d_dst_ptrs: DEVICE arrays of block pointers,
 * 8-byte aligned; every block `len` bytes, 16-byte aligned). n in [1, 256].
 * The sources of a CL repair are ecw_repair_sources' blocks. */
int ecw_xor_reduce_ptrs_dev(int device, int stripes, int n, const uint8_t* const* d_src_ptrs,
                            uint8_t* const* d_dst_ptrs, size_t len, void* stream);
/* target = XOR of n device blocks (the arithmetic of decode / partial decode
 * / relayer stage for any fan-in); n in [1, 256]. */
int ecw_xor_reduce_dev(int device, const uint8_t* const* d_src, int n, uint8_t* d_dst, size_t len,
                       void* stream);

/* ---- batched slab layout -----------------------------------------------
 * A slab holds `stripes` stripes; stripe s starts at slab + s*stripe_stride,
 * block b of a stripe at + b*block_stride. Block order inside a stripe is
 * [D_0..D_{k-1}, G_0..G_{m-1}, L_0..L_{g-1}] (ChunkGenerator.java:51-103
 * naming order). Strides must be multiples of 16; padding the block stride
 * (e.g. B + 4 KiB) spreads the k concurrent row streams over HBM channels. */
/* Encode every stripe of the slab: reads D blocks, writes G and L blocks. */
int ecw_encode_batch_dev(ecw_codec* codec, uint8_t* d_slab, size_t block_stride,
                         size_t stripe_stride, int stripes, size_t len, void* stream);
/* The same encode with data and parity blocks in separate strided regions
 * (ISA-L's separate data / coding arrays, isal:include/erasure_code.h:98, as
 * strided batches): data block j of stripe s at
 * d_data + s*data_stripe_stride + j*data_block_stride, parity block i
 * ([G_0..G_{m-1}, L_0..L_{g-1}]) at d_parity + s*parity_stripe_stride +
 * i*parity_block_stride. The regions must not overlap. Within a region the
 * stripes follow one another (stripe stride >= the stripe's extent) or are
 * interleaved inside every block (stripe stride >= len and block stride >=
 * (stripes-1)*stripe stride + len: e.g. the column pieces of one stripe of
 * whole blocks, each encoded as a stripe of its own). With 4 KiB "stripes"
 * (block stride 4096, stripe stride k*4096) it encodes a tiled layout in
 * which every 4 KiB column of the k data blocks is contiguous. */
int ecw_encode_batch_split_dev(ecw_codec* codec, const uint8_t* d_data, size_t data_block_stride,
                               size_t data_stripe_stride, uint8_t* d_parity, size_t parity_block_stride,
                               size_t parity_stripe_stride, int stripes, size_t len, void* stream);
/* Repair block `lost_block` (slab block index, D or L; G is "not yet" in the
 * reference, ClMetadataManager.java:179-182) of every stripe into
 * d_out + s*out_stride, as the XOR of its surviving group members. */
int ecw_repair_batch_dev(ecw_codec* codec, const uint8_t* d_slab, size_t block_stride,
                         size_t stripe_stride, int stripes, int lost_block, uint8_t* d_out,
                         size_t out_stride, size_t len, void* stream);
/* The same repair on the split layout of ecw_encode_batch_split_dev
 * (`lost_block` is still a stripe block index: D_j = j, L_t = k + m + t). */
int ecw_repair_batch_split_dev(ecw_codec* codec, const uint8_t* d_data, size_t data_block_stride,
                               size_t data_stripe_stride, const uint8_t* d_parity, size_t parity_block_stride,
                               size_t parity_stripe_stride, int stripes, int lost_block, uint8_t* d_out,
                               size_t out_stride, size_t len, void* stream);
/* The slab block indices whose XOR rebuilds `lost_block` (a10: the r
 * surviving members of its local group). Writes up to `cap` indices into
 * `out_blocks`, returns the count (>0) or a negative ecw_status. */
int ecw_repair_sources(const ecw_codec* codec, int lost_block, int* out_blocks, int cap);

/* ---- synthetic data ------------------------------------------------------
 * Counter-based generator used by tests and the bench (not part of the
 * codec): byte i of block `block` of stripe `stripe` is byte (i % 8) of
 *   w = mix64(key + (i/8) * 0x9E3779B97F4A7C15),
 *   key = mix64(seed + 0x9E3779B97F4A7C15 * (1 + stripe * 65536 + block)),
 * mix64 = splitmix64's finaliser. Fills `len` bytes of each of `nblocks`
 * blocks (block index b0 + i at d_dst + i*block_stride) for every stripe
 * s0 + s at + s*stripe_stride. */
int ecw_fill_random_dev(int device, uint8_t* d_dst, size_t block_stride, size_t stripe_stride,
                        int stripes, int nblocks, size_t len, uint64_t seed, int s0, int b0,
                        void* stream);
/* The same generator for blocks stored in column pieces (the tiled slab) or
 * as a column slice (a column-sharded rank): byte i of a block is byte
 * `offset` + i of its stream and lands at
 *   d_dst + s*stripe_stride + b*block_stride + (i / piece)*piece_stride + i % piece,
 * so a block holds the same bytes in every layout. piece, piece_stride and
 * offset are multiples of 16 (piece >= len: one contiguous block). */
int ecw_fill_random_pieces_dev(int device, uint8_t* d_dst, size_t block_stride, size_t stripe_stride,
                               int stripes, int nblocks, size_t len, size_t piece, size_t piece_stride,
                               size_t offset, uint64_t seed, int s0, int b0, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ECWIDE_H_ */
