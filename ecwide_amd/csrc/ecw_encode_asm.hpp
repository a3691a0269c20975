// Hand-scheduled encode of ONE full column tile (gfx950 / CDNA4), used by
// encode_kernel_asm for every encode pass (slab or pointer mode; <= 4 global rows
// below, 5-8 rows in the ECW2_* variant and 9-16 rows in the ECW4_* variant
// further down).
//
// Same arithmetic as encode_tile() in ecw_kernels.hip (ISA-L's 4-bit split
// GF(2^8) products, gf_vect_mul_init, isal:erasure_code/ec_base.c:157-262,
// with the tables of all rows of the pass packed into one LDS entry), but the
// row loop is written out so that every wait is explicit:
//
//   * two-slot register ring: row j+2 is loaded into the slot row j is
//     consumed from, and each consumption waits with vmcnt(1) -- exactly the
//     one newer ring load may stay in flight. Local-parity stores issued in
//     between do not break the count: loads return in order, so vmcnt(1)
//     with extra stores outstanding can only wait longer, never too little.
//     (Compiled from C++, any store in the row loop makes LLVM's waitcnt pass
//     fall back to vmcnt(0) at the loop head, i.e. drain the ring every two
//     rows; that cost ~4 % of encode time at k=128.)
//     With the write window on (whole-block layouts) the <= 4-row tile keeps a
//     third slot in flight (ECW_TILE_ASM3, vmcnt(2); ecw_tuning.hpp ECW_ASM_RING3).
//   * per row: the 32 table lookups are issued in two alternating sets of 8
//     (ds_read_b32 into the address register itself), each set folded into
//     the packed accumulators with v_bitop3 (xor3) while the next is in
//     flight (lgkmcnt(8));
//   * local parities: XOR of the group's rows in v[28:31], stored with a
//     global_store at the group's last row (all-zero in ECWide-C literal
//     mode, still written);
//   * global parities: v_perm byte transpose of the 16 packed accumulators,
//     one dwordx4 store per output row.
//
// Fixed registers (all declared clobbered; 57 VGPRs, 78 when parking):
//   v[4:7] ring slot A, v[8:11] ring slot B, v[12:27] packed accumulators
//   (byte column c of the lane's 16 in v[12+c]), v[28:31] local parity,
//   v32 table-record high byte, v33 nibble mask, v34/v35 nibble words,
//   v[36:39] output row, v40 column offset, v[41:48] / v[49:56] lookup sets.
//   s[40:41] next row to load, s[42:43] current local block, s44 row index,
//   s45 end of the current group, s46 LDS table record of the row, s47/s48
//   record high/low bytes, s49 scratch, s[50:53] v_perm selectors, s[54:55]
//   global output row, s56 output index, s57/s58 transpose selectors,
//   s59 finished groups, s60/s61/s62 pointer-table offsets (TAB);
//   v[58:77] parked local parities (tuples start on
//   even registers on gfx950).
#pragma once


// nibble words of data dword W (lo = (W<<2)&0x3C.. | rec.lo, hi = (W>>2)&..),
// then the 8 lookup addresses (record.hi << 8 | nibble*4) into set A0..A7
#define ECW_DW_ADDR(W, A0, A1, A2, A3, A4, A5, A6, A7) \
  "v_lshlrev_b32 v34, 2, " W "\n\t"                    \
  "v_lshrrev_b32 v35, 2, " W "\n\t"                    \
  "v_and_or_b32 v34, v34, v33, s48\n\t"                \
  "v_and_or_b32 v35, v35, v33, s48\n\t"                \
  "v_perm_b32 " A0 ", v32, v34, s50\n\t"               \
  "v_perm_b32 " A1 ", v32, v35, s50\n\t"               \
  "v_perm_b32 " A2 ", v32, v34, s51\n\t"               \
  "v_perm_b32 " A3 ", v32, v35, s51\n\t"               \
  "v_perm_b32 " A4 ", v32, v34, s52\n\t"               \
  "v_perm_b32 " A5 ", v32, v35, s52\n\t"               \
  "v_perm_b32 " A6 ", v32, v34, s53\n\t"               \
  "v_perm_b32 " A7 ", v32, v35, s53\n\t"

// lo-nibble products at +0, hi-nibble products at +64 of the record
#define ECW_DW_READ(A0, A1, A2, A3, A4, A5, A6, A7) \
  "ds_read_b32 " A0 ", " A0 "\n\t"                   \
  "ds_read_b32 " A1 ", " A1 " offset:64\n\t"         \
  "ds_read_b32 " A2 ", " A2 "\n\t"                   \
  "ds_read_b32 " A3 ", " A3 " offset:64\n\t"         \
  "ds_read_b32 " A4 ", " A4 "\n\t"                   \
  "ds_read_b32 " A5 ", " A5 " offset:64\n\t"         \
  "ds_read_b32 " A6 ", " A6 "\n\t"                   \
  "ds_read_b32 " A7 ", " A7 " offset:64\n\t"

#define ECW_DW_FOLD(C0, C1, C2, C3, A0, A1, A2, A3, A4, A5, A6, A7) \
  "v_bitop3_b32 " C0 ", " C0 ", " A0 ", " A1 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " C1 ", " C1 ", " A2 ", " A3 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " C2 ", " C2 ", " A4 ", " A5 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " C3 ", " C3 ", " A6 ", " A7 " bitop3:0x96\n\t"

#define ECW_ADDR_X(W) ECW_DW_ADDR(W, "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48")
#define ECW_ADDR_Y(W) ECW_DW_ADDR(W, "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56")
#define ECW_READ_X ECW_DW_READ("v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48")
#define ECW_READ_Y ECW_DW_READ("v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56")
#define ECW_FOLD_X(C0, C1, C2, C3) ECW_DW_FOLD(C0, C1, C2, C3, "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48")
#define ECW_FOLD_Y(C0, C1, C2, C3) ECW_DW_FOLD(C0, C1, C2, C3, "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56")

// One data row from ring slot R0..R3 (s46 = its LDS table record): GF
// products into the accumulators, XOR into the local parity (XL = 1).
// Software-pipelined across rows: the row's last lookup set (Y, from R3) is
// left in flight and folded after the next row's first set has been issued,
// so the LDS lookups never drain at a row boundary -- not behind the next
// ring slot's vmcnt wait either (ECW_ROW_DRAIN folds it after the last row;
// the Y set is zero at the start of a tile, so the first fold is a no-op).
// A row is split where its ring slot's registers are last read (ECW_ROW_PRE:
// every address computed and the local XOR done; ECW_ROW_POST: the last
// folds), so in slab mode the slot's next load is issued between the two.
#define ECW_ROW_PRE(R0, R1, R2, R3, XL)                               \
  "s_lshr_b32 s47, s46, 8\n\t"                                        \
  "s_and_b32 s48, s46, 0xff\n\t"                                      \
  "s_mul_i32 s48, s48, 0x01010101\n\t"                                \
  "v_mov_b32 v32, s47\n\t"                                            \
  ECW_ADDR_X(R0) ECW_READ_X                                           \
  "s_waitcnt lgkmcnt(8)\n\t"                                          \
  ECW_FOLD_Y("v24", "v25", "v26", "v27")                              \
  ECW_ADDR_Y(R1) ECW_READ_Y                                           \
  "s_waitcnt lgkmcnt(8)\n\t"                                          \
  ECW_FOLD_X("v12", "v13", "v14", "v15")                              \
  ECW_ADDR_X(R2) ECW_READ_X                                           \
  "s_waitcnt lgkmcnt(8)\n\t"                                          \
  ECW_FOLD_Y("v16", "v17", "v18", "v19")                              \
  ECW_ADDR_Y(R3) ECW_READ_Y                                           \
  ECW_LACC_##XL(R0, R1, R2, R3)                                       \
  "s_add_u32 s46, s46, 128\n\t"
#define ECW_ROW_POST                                                  \
  "s_waitcnt lgkmcnt(8)\n\t"                                          \
  ECW_FOLD_X("v20", "v21", "v22", "v23")
#define ECW_ROW_DRAIN "s_waitcnt lgkmcnt(0)\n\t" ECW_FOLD_Y("v24", "v25", "v26", "v27")
#define ECW_ROW_YZERO                                                 \
  "v_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\tv_mov_b32 v52, 0\n\t" \
  "v_mov_b32 v53, 0\n\tv_mov_b32 v54, 0\n\tv_mov_b32 v55, 0\n\tv_mov_b32 v56, 0\n\t"
#define ECW_ROW(R0, R1, R2, R3, XL) ECW_ROW_PRE(R0, R1, R2, R3, XL) ECW_ROW_POST

#define ECW_LACC_0(R0, R1, R2, R3)
#define ECW_LACC_1(R0, R1, R2, R3)     \
  "v_xor_b32 v28, v28, " R0 "\n\t"     \
  "v_xor_b32 v29, v29, " R1 "\n\t"     \
  "v_xor_b32 v30, v30, " R2 "\n\t"     \
  "v_xor_b32 v31, v31, " R3 "\n\t"

// End of the local group at row s44 (0-based)? Store the local parity,
// advance to the next local block and group. ZL = 1: reset the XOR.
#define ECW_BOUNDARY_NONE
#define ECW_BOUNDARY(ZL, MODE)                            \
  "s_add_u32 s49, s44, 1\n\t"                             \
  "s_cmp_eq_u32 s49, s45\n\t"                             \
  "s_cbranch_scc0 20f\n\t"                                \
  ECW_LPTR_GET_##MODE                                     \
  ECW_ASM_LSTORE                                          \
  ECW_LPTR_NEXT_##MODE                                    \
  "s_add_u32 s45, s45, %[r]\n\t"                          \
  "s_min_u32 s45, s45, %[k]\n\t"                          \
  "s_nop 1\n\t"                                           \
  ECW_LRESET_##ZL                                         \
  "20:\n\t"
// Parked variant (<= 5 groups): the finished local parity is copied into
// v[58+4t:61+4t] and all locals are stored at the end of the tile, next to
// the global rows. Mid-tile stores measured ~9 % of encode time at k=128
// (3.7 % of the bytes): writes scattered between the row reads cost the
// DRAM far more than the same writes issued together.
#define ECW_PARK(T, V0, V1, V2, V3, NEXT)                                   \
  "s_cmp_eq_u32 s59, " #T "\n\t"                                            \
  "s_cbranch_scc0 " #NEXT "f\n\t"                                           \
  "v_mov_b32 " V0 ", v28\n\tv_mov_b32 " V1 ", v29\n\t"                       \
  "v_mov_b32 " V2 ", v30\n\tv_mov_b32 " V3 ", v31\n\t"                       \
  "s_branch 26f\n\t" #NEXT ":\n\t"
#define ECW_BOUNDARY_PARK                                   \
  "s_add_u32 s49, s44, 1\n\t"                               \
  "s_cmp_eq_u32 s49, s45\n\t"                               \
  "s_cbranch_scc0 20f\n\t"                                  \
  ECW_PARK(0, "v58", "v59", "v60", "v61", 21)               \
  ECW_PARK(1, "v62", "v63", "v64", "v65", 22)               \
  ECW_PARK(2, "v66", "v67", "v68", "v69", 23)               \
  ECW_PARK(3, "v70", "v71", "v72", "v73", 24)               \
  ECW_PARK(4, "v74", "v75", "v76", "v77", 25)               \
  "26:\n\t"                                                 \
  "s_add_u32 s59, s59, 1\n\t"                               \
  "s_add_u32 s45, s45, %[r]\n\t"                            \
  "s_min_u32 s45, s45, %[k]\n\t"                            \
  ECW_LRESET_1                                              \
  "20:\n\t"
// store parked local t (if t < number of groups) and advance the block
#define ECW_UNPARK(T, V, MODE)                                              \
  "s_cmp_le_u32 s59, " #T "\n\t"                                            \
  "s_cbranch_scc1 27f\n\t"                                                  \
  ECW_LPTR_GET_##MODE                                                       \
  ECW_ASM_GSTORE(V, "s[42:43]")                                             \
  ECW_LPTR_NEXT_##MODE
#define ECW_STORE_PARKED(MODE)                                              \
  ECW_LPTR_INIT_##MODE                                                      \
  ECW_UNPARK(0, "v[58:61]", MODE) ECW_UNPARK(1, "v[62:65]", MODE)           \
  ECW_UNPARK(2, "v[66:69]", MODE) ECW_UNPARK(3, "v[70:73]", MODE)           \
  ECW_UNPARK(4, "v[74:77]", MODE)                                           \
  "27:\n\t"

// ECWide-C literal mode (every L block is zeros): the rows only count the
// finished groups, and the end of the tile stores v[28:31] (zero throughout)
// once per group -- the same end-of-tile placement as the parked parities,
// for any number of groups.
#define ECW_BOUNDARY_COUNT                                  \
  "s_add_u32 s49, s44, 1\n\t"                               \
  "s_cmp_eq_u32 s49, s45\n\t"                               \
  "s_cbranch_scc0 20f\n\t"                                  \
  "s_add_u32 s59, s59, 1\n\t"                               \
  "s_add_u32 s45, s45, %[r]\n\t"                            \
  "s_min_u32 s45, s45, %[k]\n\t"                            \
  "20:\n\t"
#define ECW_STORE_ZEROS(MODE)                                               \
  ECW_LPTR_INIT_##MODE                                                      \
  "28:\n\t"                                                                 \
  "s_cmp_eq_u32 s59, 0\n\t"                                                 \
  "s_cbranch_scc1 29f\n\t"                                                  \
  ECW_LPTR_GET_##MODE                                                       \
  ECW_ASM_GSTORE("v[28:31]", "s[42:43]")                                    \
  ECW_LPTR_NEXT_##MODE                                                      \
  "s_sub_u32 s59, s59, 1\n\t"                                               \
  "s_branch 28b\n\t"                                                        \
  "29:\n\t"

// Block pointers. SLAB: %[row0] / %[lrow0] / %[grow0] are the first data,
// local and global blocks; data blocks are %[bslo]/%[bshi] apart, parity
// blocks %[pbslo]/%[pbshi]. TAB (pointer mode):
// they are the addresses of pointer tables in the kernel arguments
// (PtrRows::src, &dst[nrows], &dst[0]), and every block pointer is an
// s_load. The row pointer for the next ring load is fetched right after the
// previous load and is ready behind the next row's lgkmcnt(0); the counted
// lgkmcnt waits inside a row stay correct with an s_load outstanding (LDS
// returns in order; an extra outstanding op only makes them wait longer).
#define ECW_ROWPTR_INIT_SLAB "s_mov_b64 s[40:41], %[row0]\n\t"
#define ECW_ROWPTR_INIT_TAB "s_load_dwordx2 s[40:41], %[row0], 0x0\n\ts_mov_b32 s60, 8\n\ts_waitcnt lgkmcnt(0)\n\t"
#define ECW_NEXTROW_SLAB "s_add_u32 s40, s40, %[bslo]\n\ts_addc_u32 s41, s41, %[bshi]\n\t"
// before a ring load: the row pointer it uses has arrived. TAB: the s_load
// issued behind the previous ring load (the pipelined rows keep LDS lookups in
// flight, so no lgkmcnt wait inside a row implies it); SLAB: pointers are sums.
#define ECW_LDWAIT_SLAB
#define ECW_LDWAIT_TAB "s_waitcnt lgkmcnt(0)\n\t"
#define ECW_NEXTROW_TAB "s_load_dwordx2 s[40:41], %[row0], s60\n\ts_add_u32 s60, s60, 8\n\t"
#define ECW_LPTR_INIT_SLAB "s_mov_b64 s[42:43], %[lrow0]\n\t"
#define ECW_LPTR_INIT_TAB "s_mov_b32 s61, 0\n\t"
#define ECW_LPTR_GET_SLAB
#define ECW_LPTR_GET_TAB "s_load_dwordx2 s[42:43], %[lrow0], s61\n\ts_waitcnt lgkmcnt(0)\n\t"
#define ECW_LPTR_NEXT_SLAB "s_add_u32 s42, s42, %[pbslo]\n\ts_addc_u32 s43, s43, %[pbshi]\n\t"
#define ECW_LPTR_NEXT_TAB "s_add_u32 s61, s61, 8\n\t"
#define ECW_GPTR_INIT_SLAB "s_mov_b64 s[54:55], %[grow0]\n\t"
#define ECW_GPTR_INIT_TAB "s_mov_b32 s62, 0\n\t"
#define ECW_GPTR_GET_SLAB
#define ECW_GPTR_GET_TAB "s_load_dwordx2 s[54:55], %[grow0], s62\n\ts_waitcnt lgkmcnt(0)\n\t"
#define ECW_GPTR_NEXT_SLAB "s_add_u32 s54, s54, %[pbslo]\n\ts_addc_u32 s55, s55, %[pbshi]\n\t"
#define ECW_GPTR_NEXT_TAB "s_add_u32 s62, s62, 8\n\t"
#define ECW_LRESET_0
#define ECW_LRESET_1 "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\tv_mov_b32 v30, 0\n\tv_mov_b32 v31, 0\n\t"

// Write window (EncodeGeom::wwidth > 0). A tile's parity stores wait until
// the chip-wide 100 MHz constant clock (s_memrealtime: the same counter on
// every CU) is in the first `wwidth` ticks of every `wmask + 1`. HBM pays for
// each switch between reading and writing far more than for the written bytes
// (1 output row per 128 read rows costs +9 % time); gathering every
// workgroup's stores into the same short windows gives the memory long read
// runs and short write bursts. A wave waits on its own (no workgroup barrier),
// at most wmask + 1 ticks (and at most 16384 polls, whatever the clock does).
// Which layouts use it: launch_encode (ecw_kernels.hip).
#define ECW_WRITE_WINDOW                                                     \
  "s_cmp_eq_u32 %[ww], 0\n\t"                                               \
  "s_cbranch_scc1 35f\n\t"                                                  \
  "s_mov_b32 s47, 0\n\t"                                                    \
  "34:\n\t"                                                                 \
  "s_memrealtime s[48:49]\n\t"                                              \
  "s_waitcnt lgkmcnt(0)\n\t"                                                \
  "s_and_b32 s48, s48, %[wmask]\n\t"                                        \
  "s_cmp_lt_u32 s48, %[ww]\n\t"                                             \
  "s_cbranch_scc1 35f\n\t"                                                  \
  "s_add_u32 s47, s47, 1\n\t"                                               \
  "s_cmp_gt_u32 s47, 0x4000\n\t"        /* bound: never wait unboundedly */ \
  "s_cbranch_scc1 35f\n\t"                                                  \
  "s_sleep 2\n\t"                                                           \
  "s_branch 34b\n\t"                                                        \
  "35:\n\t"

// parity stores: nontemporal (+3 % encode over plain stores, round 1) at system
// scope (sc0 sc1: +0.4..0.7 % over nt alone on the tiled slab in three
// processes, +0.5 % block slab; profiles/r02_encode_store_policy_ab.log)
#define ECW_ASM_STMOD " nt sc0 sc1"
// ring loads: nontemporal, every byte is read once (+2 %, measured); nt sc1 /
// nt sc0 sc1 the same, sc0 sc1 without nt -9 % (profiles/r02_encode_load_policy_ab.log)
#define ECW_ASM_LDMOD " nt"
#define ECW_ASM_GSTORE(V, S) "global_store_dwordx4 v40, " V ", " S ECW_ASM_STMOD "\n\t"
#define ECW_ASM_LSTORE ECW_ASM_GSTORE("v[28:31]", "s[42:43]")
#define ECW_LOAD_A "global_load_dwordx4 v[4:7], v40, s[40:41]" ECW_ASM_LDMOD "\n\t"
#define ECW_LOAD_B "global_load_dwordx4 v[8:11], v40, s[40:41]" ECW_ASM_LDMOD "\n\t"
#define ECW_ROW_A(XL) ECW_ROW("v4", "v5", "v6", "v7", XL)
#define ECW_ROW_B(XL) ECW_ROW("v8", "v9", "v10", "v11", XL)
#define ECW_ROW_PRE_A(XL) ECW_ROW_PRE("v4", "v5", "v6", "v7", XL)
#define ECW_ROW_PRE_B(XL) ECW_ROW_PRE("v8", "v9", "v10", "v11", XL)
// A row whose ring slot is reloaded with the row two ahead. SLAB: the load
// goes out as soon as the slot is consumed (between PRE and POST); TAB: after
// the row, behind the wait for its row-pointer s_load (ECW_LDWAIT_TAB, which
// drains the LDS lookups too).
#define ECW_STEP_SLAB(PRE, LOAD, NEXT, BND) PRE LOAD NEXT ECW_ROW_POST BND
#define ECW_STEP_TAB(PRE, LOAD, NEXT, BND) PRE ECW_ROW_POST BND ECW_LDWAIT_TAB LOAD NEXT

// The whole tile. BND is the boundary code (ECW_BOUNDARY(ZL, MODE) or
// nothing), XL whether rows are XOR-ed into the local parity, END the code
// after the last row (parked locals), MODE SLAB or TAB.
#define ECW_TILE_ASM(BND, XL, END, MODE)                                           \
  "v_mov_b32 v40, %[col]\n\t"                                               \
  "v_mov_b32 v33, 0x3c3c3c3c\n\t"                                           \
  "s_mov_b32 s50, 0x0c0c0400\n\t"                                           \
  "s_mov_b32 s51, 0x0c0c0401\n\t"                                           \
  "s_mov_b32 s52, 0x0c0c0402\n\t"                                           \
  "s_mov_b32 s53, 0x0c0c0403\n\t"                                           \
  ECW_ROWPTR_INIT_##MODE                                                    \
  ECW_LOAD_A ECW_NEXTROW_##MODE "s_waitcnt lgkmcnt(0)\n\t"                  \
  ECW_LOAD_B ECW_NEXTROW_##MODE                                             \
  "v_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\tv_mov_b32 v15, 0\n\t" \
  "v_mov_b32 v16, 0\n\tv_mov_b32 v17, 0\n\tv_mov_b32 v18, 0\n\tv_mov_b32 v19, 0\n\t" \
  "v_mov_b32 v20, 0\n\tv_mov_b32 v21, 0\n\tv_mov_b32 v22, 0\n\tv_mov_b32 v23, 0\n\t" \
  "v_mov_b32 v24, 0\n\tv_mov_b32 v25, 0\n\tv_mov_b32 v26, 0\n\tv_mov_b32 v27, 0\n\t" \
  "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\tv_mov_b32 v30, 0\n\tv_mov_b32 v31, 0\n\t" \
  ECW_ROW_YZERO                                                             \
  "s_mov_b32 s44, 0\n\t"                                                    \
  "s_mov_b32 s59, 0\n\t"                                                    \
  "s_mov_b32 s46, %[lds]\n\t"                                               \
  ECW_LPTR_INIT_##MODE                                                      \
  "s_min_u32 s45, %[r], %[k]\n\t"                                           \
  /* main loop: rows j, j+1 while rows j+2, j+3 exist */                    \
  "10:\n\t"                                                                 \
  "s_add_u32 s49, s44, 3\n\t"                                               \
  "s_cmp_ge_u32 s49, %[k]\n\t"                                              \
  "s_cbranch_scc1 11f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW_STEP_##MODE(ECW_ROW_PRE_A(XL), ECW_LOAD_A, ECW_NEXTROW_##MODE, BND)                           \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW_STEP_##MODE(ECW_ROW_PRE_B(XL), ECW_LOAD_B, ECW_NEXTROW_##MODE, BND)                           \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_branch 10b\n\t"                                                        \
  /* 2 or 3 rows left (k - j); slot A holds row j, slot B row j+1 */        \
  "11:\n\t"                                                                 \
  "s_sub_u32 s49, %[k], s44\n\t"                                            \
  "s_cmp_eq_u32 s49, 3\n\t"                                                 \
  "s_cbranch_scc0 12f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW_STEP_##MODE(ECW_ROW_PRE_A(XL), ECW_LOAD_A, , BND)                    \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW_ROW_B(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW_ROW_A(XL) BND                                                         \
  "s_branch 13f\n\t"                                                        \
  "12:\n\t"                                                                 \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW_ROW_A(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW_ROW_B(XL) BND                                                         \
  "13:\n\t"                                                                 \
  ECW_ROW_DRAIN                                                             \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW_GLOBAL_ROWS(MODE)

// global rows: byte l of the packed accumulators -> output row l (v[36:39])
#define ECW_GLOBAL_ROWS(MODE)                                                    \
  ECW_GPTR_INIT_##MODE                                                      \
  "s_mov_b32 s56, 0\n\t"                                                    \
  "30:\n\t"                                                                 \
  "s_cmp_ge_u32 s56, %[nrows]\n\t"                                          \
  "s_cbranch_scc1 31f\n\t"                                                  \
  "s_add_u32 s49, s56, 4\n\t"                                               \
  "s_lshl_b32 s57, s49, 8\n\t"                                              \
  "s_or_b32 s57, s57, s56\n\t"                                              \
  "s_or_b32 s57, s57, 0x0c0c0000\n\t"                                       \
  "s_lshl_b32 s58, s49, 24\n\t"                                             \
  "s_lshl_b32 s49, s56, 16\n\t"                                             \
  "s_or_b32 s58, s58, s49\n\t"                                              \
  "s_or_b32 s58, s58, 0x0c0c\n\t"                                           \
  "v_perm_b32 v34, v13, v12, s57\n\t"                                       \
  "v_perm_b32 v35, v15, v14, s58\n\t"                                       \
  "v_or_b32 v36, v34, v35\n\t"                                              \
  "v_perm_b32 v34, v17, v16, s57\n\t"                                       \
  "v_perm_b32 v35, v19, v18, s58\n\t"                                       \
  "v_or_b32 v37, v34, v35\n\t"                                              \
  "v_perm_b32 v34, v21, v20, s57\n\t"                                       \
  "v_perm_b32 v35, v23, v22, s58\n\t"                                       \
  "v_or_b32 v38, v34, v35\n\t"                                              \
  "v_perm_b32 v34, v25, v24, s57\n\t"                                       \
  "v_perm_b32 v35, v27, v26, s58\n\t"                                       \
  "v_or_b32 v39, v34, v35\n\t"                                              \
  ECW_GPTR_GET_##MODE                                                       \
  ECW_ASM_GSTORE("v[36:39]", "s[54:55]")                                    \
  "s_nop 1\n\t"                                                             \
  ECW_GPTR_NEXT_##MODE                                                      \
  "s_add_u32 s56, s56, 1\n\t"                                               \
  "s_branch 30b\n\t"                                                        \
  "31:"

// Three-slot ring (kAsmRing3, k >= 3): slot C is v[36:39], the output-row
// registers, which the row loop does not use; rows j, j+1, j+2 are in flight
// and each consumption waits with vmcnt(2). Same rows, boundaries and stores
// as ECW_TILE_ASM; 1 KiB more read in flight per wave at no register cost.
#define ECW_LOAD_C "global_load_dwordx4 v[36:39], v40, s[40:41]" ECW_ASM_LDMOD "\n\t"
#define ECW_ROW_C(XL) ECW_ROW("v36", "v37", "v38", "v39", XL)
#define ECW_ROW_PRE_C(XL) ECW_ROW_PRE("v36", "v37", "v38", "v39", XL)
// The three-slot row loop of every asm tile (P = ECW / ECW2 / ECW4: that tile's
// STEP / ROW / ROW_DRAIN macros; slot C = v[36:39], idle until the global rows):
// rows j, j+1, j+2 in flight, each consumption behind vmcnt(2); the tail takes the
// last 3, 4 or 5 rows. Needs k >= 3.
#define ECW_RING3_ROWS(P, BND, XL, MODE)                                            \
  /* main loop: rows j..j+2 while rows j+3..j+5 exist */                    \
  "10:\n\t"                                                                 \
  "s_add_u32 s49, s44, 5\n\t"                                               \
  "s_cmp_ge_u32 s49, %[k]\n\t"                                              \
  "s_cbranch_scc1 11f\n\t"                                                  \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_A(XL), ECW_LOAD_A, ECW_NEXTROW_##MODE, BND)   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_B(XL), ECW_LOAD_B, ECW_NEXTROW_##MODE, BND)   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_C(XL), ECW_LOAD_C, ECW_NEXTROW_##MODE, BND)   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_branch 10b\n\t"                                                        \
  /* 3, 4 or 5 rows left (k - j); slots A, B, C hold rows j, j+1, j+2 */    \
  "11:\n\t"                                                                 \
  "s_sub_u32 s49, %[k], s44\n\t"                                            \
  "s_cmp_eq_u32 s49, 3\n\t"                                                 \
  "s_cbranch_scc1 12f\n\t"                                                  \
  "s_cmp_eq_u32 s49, 4\n\t"                                                 \
  "s_cbranch_scc1 14f\n\t"                                                  \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_A(XL), ECW_LOAD_A, ECW_NEXTROW_##MODE, BND)   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_B(XL), ECW_LOAD_B, , BND)                     \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_ROW_C(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  P##_ROW_A(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  P##_ROW_B(XL) BND                                                         \
  "s_branch 13f\n\t"                                                        \
  "14:\n\t"                                                                 \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_STEP_##MODE(P##_ROW_PRE_A(XL), ECW_LOAD_A, , BND)                     \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_ROW_B(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  P##_ROW_C(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  P##_ROW_A(XL) BND                                                         \
  "s_branch 13f\n\t"                                                        \
  "12:\n\t"                                                                 \
  "s_waitcnt vmcnt(2)\n\t"                                                  \
  P##_ROW_A(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  P##_ROW_B(XL) BND                                                         \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  P##_ROW_C(XL) BND                                                         \
  "13:\n\t"                                                                 \
  P##_ROW_DRAIN

#define ECW_TILE_ASM3(BND, XL, END, MODE)                                          \
  "v_mov_b32 v40, %[col]\n\t"                                               \
  "v_mov_b32 v33, 0x3c3c3c3c\n\t"                                           \
  "s_mov_b32 s50, 0x0c0c0400\n\t"                                           \
  "s_mov_b32 s51, 0x0c0c0401\n\t"                                           \
  "s_mov_b32 s52, 0x0c0c0402\n\t"                                           \
  "s_mov_b32 s53, 0x0c0c0403\n\t"                                           \
  ECW_ROWPTR_INIT_##MODE                                                    \
  ECW_LOAD_A ECW_NEXTROW_##MODE "s_waitcnt lgkmcnt(0)\n\t"                  \
  ECW_LOAD_B ECW_NEXTROW_##MODE "s_waitcnt lgkmcnt(0)\n\t"                  \
  ECW_LOAD_C ECW_NEXTROW_##MODE                                             \
  "v_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\tv_mov_b32 v15, 0\n\t" \
  "v_mov_b32 v16, 0\n\tv_mov_b32 v17, 0\n\tv_mov_b32 v18, 0\n\tv_mov_b32 v19, 0\n\t" \
  "v_mov_b32 v20, 0\n\tv_mov_b32 v21, 0\n\tv_mov_b32 v22, 0\n\tv_mov_b32 v23, 0\n\t" \
  "v_mov_b32 v24, 0\n\tv_mov_b32 v25, 0\n\tv_mov_b32 v26, 0\n\tv_mov_b32 v27, 0\n\t" \
  "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\tv_mov_b32 v30, 0\n\tv_mov_b32 v31, 0\n\t" \
  ECW_ROW_YZERO                                                             \
  "s_mov_b32 s44, 0\n\t"                                                    \
  "s_mov_b32 s59, 0\n\t"                                                    \
  "s_mov_b32 s46, %[lds]\n\t"                                               \
  ECW_LPTR_INIT_##MODE                                                      \
  "s_min_u32 s45, %[r], %[k]\n\t"                                           \
  ECW_RING3_ROWS(ECW, BND, XL, MODE)                                        \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW_GLOBAL_ROWS(MODE)

#define ECW_TILE_OPERANDS                                                          \
  : : [row0] "s"(row0), [lrow0] "s"(lrow0), [grow0] "s"(grow0), [bslo] "s"(bslo), \
    [bshi] "s"(bshi), [pbslo] "s"(pbslo), [pbshi] "s"(pbshi), [k] "s"(k), [r] "s"(r),  \
    [nrows] "s"(nrows), [lds] "s"(lds), [wmask] "s"(wmask), [ww] "s"(ww),          \
    [col] "v"(col)                                                                 \
  : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18",  \
    "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32",  \
    "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46",  \
    "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "s40", "s41", "s42", "s43", \
    "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57",  \
    "s58", "s59", "s60", "s61", "s62", "scc", "memory"

#define ECW_TILE_OPERANDS_PARK                                                     \
  ECW_TILE_OPERANDS, "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", \
    "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77"

// ---------------------------------------------------------------------------
// 5-8 global rows (NW = 2): the same tile with one u64 table entry per nibble
// (rows 0-3 in the low dword, 4-7 in the high one; records of 256 B, hi- and
// lo-nibble entries interleaved: hi of nibble n at +16n, lo at +16n + 8) and a
// second bank of packed accumulators. The interleaving makes a hi address the
// data byte's high nibble as it stands, so the nibble words cost one shift
// instead of two; byte 0's addresses are built with v_bitop3 (2 cycles) instead
// of v_perm (4): (word & 0xff) | the record address without its low byte.
// Registers as above except: v33 = 0xF0F0F0F0 (nibble * 16), v41 = 0xff, s63
// = the record address with its low byte cleared, lookup sets v[42:57] /
// v[58:73] (eight even-aligned pairs each, the address in the low register of
// its pair), accumulators of rows 4-7 in v[74:89], parked local parities in
// v[90:109].
#define ECW2_DW_ADDR(W, A0, A1, A2, A3, A4, A5, A6, A7) \
  "v_lshlrev_b32 v34, 4, " W "\n\t"                     \
  "v_bitop3_b32 v34, v34, v33, s48 bitop3:0xea\n\t"     \
  "v_bitop3_b32 v35, " W ", v33, s48 bitop3:0xea\n\t"   \
  "v_bitop3_b32 " A0 ", v34, v41, s63 bitop3:0xea\n\t"  \
  "v_bitop3_b32 " A1 ", v35, v41, s63 bitop3:0xea\n\t"  \
  "v_perm_b32 " A2 ", v32, v34, s51\n\t"                \
  "v_perm_b32 " A3 ", v32, v35, s51\n\t"                \
  "v_perm_b32 " A4 ", v32, v34, s52\n\t"                \
  "v_perm_b32 " A5 ", v32, v35, s52\n\t"                \
  "v_perm_b32 " A6 ", v32, v34, s53\n\t"                \
  "v_perm_b32 " A7 ", v32, v35, s53\n\t"
#define ECW2_ADDR_X(W) ECW2_DW_ADDR(W, "v42", "v44", "v46", "v48", "v50", "v52", "v54", "v56")
#define ECW2_ADDR_Y(W) ECW2_DW_ADDR(W, "v58", "v60", "v62", "v64", "v66", "v68", "v70", "v72")
#define ECW2_READ_X                                 \
  "ds_read_b64 v[42:43], v42 offset:8\n\t"          \
  "ds_read_b64 v[44:45], v44\n\t"                   \
  "ds_read_b64 v[46:47], v46 offset:8\n\t"          \
  "ds_read_b64 v[48:49], v48\n\t"                   \
  "ds_read_b64 v[50:51], v50 offset:8\n\t"          \
  "ds_read_b64 v[52:53], v52\n\t"                   \
  "ds_read_b64 v[54:55], v54 offset:8\n\t"          \
  "ds_read_b64 v[56:57], v56\n\t"
#define ECW2_READ_Y                                 \
  "ds_read_b64 v[58:59], v58 offset:8\n\t"          \
  "ds_read_b64 v[60:61], v60\n\t"                   \
  "ds_read_b64 v[62:63], v62 offset:8\n\t"          \
  "ds_read_b64 v[64:65], v64\n\t"                   \
  "ds_read_b64 v[66:67], v66 offset:8\n\t"          \
  "ds_read_b64 v[68:69], v68\n\t"                   \
  "ds_read_b64 v[70:71], v70 offset:8\n\t"          \
  "ds_read_b64 v[72:73], v72\n\t"
// byte b of the dword: lo-nibble pair (L, L+1), hi-nibble pair (H, H+1) into
// accumulators C (rows 0-3) and D (rows 4-7)
#define ECW2_FOLD1(C, D, L, L1, H, H1)                    \
  "v_bitop3_b32 " C ", " C ", " L ", " H " bitop3:0x96\n\t"  \
  "v_bitop3_b32 " D ", " D ", " L1 ", " H1 " bitop3:0x96\n\t"
#define ECW2_FOLD_X(C0, C1, C2, C3, D0, D1, D2, D3)        \
  ECW2_FOLD1(C0, D0, "v42", "v43", "v44", "v45")           \
  ECW2_FOLD1(C1, D1, "v46", "v47", "v48", "v49")           \
  ECW2_FOLD1(C2, D2, "v50", "v51", "v52", "v53")           \
  ECW2_FOLD1(C3, D3, "v54", "v55", "v56", "v57")
#define ECW2_FOLD_Y(C0, C1, C2, C3, D0, D1, D2, D3)        \
  ECW2_FOLD1(C0, D0, "v58", "v59", "v60", "v61")           \
  ECW2_FOLD1(C1, D1, "v62", "v63", "v64", "v65")           \
  ECW2_FOLD1(C2, D2, "v66", "v67", "v68", "v69")           \
  ECW2_FOLD1(C3, D3, "v70", "v71", "v72", "v73")
// Pipelined across rows as ECW_ROW_PRE / ECW_ROW_POST above: the row's last
// lookup set (Y, from R3) is folded after the next row's first set is issued.
#define ECW2_ROW_PRE(R0, R1, R2, R3, XL)                                               \
  "s_lshr_b32 s47, s46, 8\n\t"                                                         \
  "s_and_b32 s48, s46, 0xff\n\t"                                                       \
  "s_andn2_b32 s63, s46, 0xff\n\t"                                                     \
  "s_mul_i32 s48, s48, 0x01010101\n\t"                                                 \
  "v_mov_b32 v32, s47\n\t"                                                             \
  ECW2_ADDR_X(R0) ECW2_READ_X                                                          \
  "s_waitcnt lgkmcnt(8)\n\t"                                                           \
  ECW2_FOLD_Y("v24", "v25", "v26", "v27", "v86", "v87", "v88", "v89")                 \
  ECW2_ADDR_Y(R1) ECW2_READ_Y                                                          \
  "s_waitcnt lgkmcnt(8)\n\t"                                                           \
  ECW2_FOLD_X("v12", "v13", "v14", "v15", "v74", "v75", "v76", "v77")                 \
  ECW2_ADDR_X(R2) ECW2_READ_X                                                          \
  "s_waitcnt lgkmcnt(8)\n\t"                                                           \
  ECW2_FOLD_Y("v16", "v17", "v18", "v19", "v78", "v79", "v80", "v81")                 \
  ECW2_ADDR_Y(R3) ECW2_READ_Y                                                          \
  ECW_LACC_##XL(R0, R1, R2, R3)                                                        \
  "s_add_u32 s46, s46, 256\n\t"
#define ECW2_ROW_POST                                                                  \
  "s_waitcnt lgkmcnt(8)\n\t"                                                           \
  ECW2_FOLD_X("v20", "v21", "v22", "v23", "v82", "v83", "v84", "v85")
#define ECW2_ROW_DRAIN \
  "s_waitcnt lgkmcnt(0)\n\t" ECW2_FOLD_Y("v24", "v25", "v26", "v27", "v86", "v87", "v88", "v89")
#define ECW2_ROW_YZERO                                                                 \
  "v_mov_b32 v58, 0\n\tv_mov_b32 v59, 0\n\tv_mov_b32 v60, 0\n\tv_mov_b32 v61, 0\n\t"     \
  "v_mov_b32 v62, 0\n\tv_mov_b32 v63, 0\n\tv_mov_b32 v64, 0\n\tv_mov_b32 v65, 0\n\t"     \
  "v_mov_b32 v66, 0\n\tv_mov_b32 v67, 0\n\tv_mov_b32 v68, 0\n\tv_mov_b32 v69, 0\n\t"     \
  "v_mov_b32 v70, 0\n\tv_mov_b32 v71, 0\n\tv_mov_b32 v72, 0\n\tv_mov_b32 v73, 0\n\t"
#define ECW2_ROW(R0, R1, R2, R3, XL) ECW2_ROW_PRE(R0, R1, R2, R3, XL) ECW2_ROW_POST
#define ECW2_ROW_A(XL) ECW2_ROW("v4", "v5", "v6", "v7", XL)
#define ECW2_ROW_B(XL) ECW2_ROW("v8", "v9", "v10", "v11", XL)
#define ECW2_ROW_PRE_A(XL) ECW2_ROW_PRE("v4", "v5", "v6", "v7", XL)
#define ECW2_ROW_PRE_B(XL) ECW2_ROW_PRE("v8", "v9", "v10", "v11", XL)
// as ECW_STEP_* for the 8-row rows
#define ECW2_STEP_SLAB(PRE, LOAD, NEXT, BND) PRE LOAD NEXT ECW2_ROW_POST BND
#define ECW2_STEP_TAB(PRE, LOAD, NEXT, BND) PRE ECW2_ROW_POST BND ECW_LDWAIT_TAB LOAD NEXT

#define ECW2_BOUNDARY_PARK                                  \
  "s_add_u32 s49, s44, 1\n\t"                               \
  "s_cmp_eq_u32 s49, s45\n\t"                               \
  "s_cbranch_scc0 20f\n\t"                                  \
  ECW_PARK(0, "v90", "v91", "v92", "v93", 21)               \
  ECW_PARK(1, "v94", "v95", "v96", "v97", 22)               \
  ECW_PARK(2, "v98", "v99", "v100", "v101", 23)             \
  ECW_PARK(3, "v102", "v103", "v104", "v105", 24)           \
  ECW_PARK(4, "v106", "v107", "v108", "v109", 25)           \
  "26:\n\t"                                                 \
  "s_add_u32 s59, s59, 1\n\t"                               \
  "s_add_u32 s45, s45, %[r]\n\t"                            \
  "s_min_u32 s45, s45, %[k]\n\t"                            \
  ECW_LRESET_1                                              \
  "20:\n\t"
#define ECW2_STORE_PARKED(MODE)                                             \
  ECW_LPTR_INIT_##MODE                                                      \
  ECW_UNPARK(0, "v[90:93]", MODE) ECW_UNPARK(1, "v[94:97]", MODE)           \
  ECW_UNPARK(2, "v[98:101]", MODE) ECW_UNPARK(3, "v[102:105]", MODE)        \
  ECW_UNPARK(4, "v[106:109]", MODE)                                         \
  "27:\n\t"

// byte s49 of the packed accumulators C0..C15 -> v[36:39] (selectors s57/s58)
#define ECW2_TRANSPOSE(C0, C1, C2, C3, C4, C5, C6, C7, C8, C9, C10, C11, C12, C13, C14, C15) \
  "v_perm_b32 v34, " C1 ", " C0 ", s57\n\t"                                 \
  "v_perm_b32 v35, " C3 ", " C2 ", s58\n\t"                                 \
  "v_or_b32 v36, v34, v35\n\t"                                              \
  "v_perm_b32 v34, " C5 ", " C4 ", s57\n\t"                                 \
  "v_perm_b32 v35, " C7 ", " C6 ", s58\n\t"                                 \
  "v_or_b32 v37, v34, v35\n\t"                                              \
  "v_perm_b32 v34, " C9 ", " C8 ", s57\n\t"                                 \
  "v_perm_b32 v35, " C11 ", " C10 ", s58\n\t"                               \
  "v_or_b32 v38, v34, v35\n\t"                                              \
  "v_perm_b32 v34, " C13 ", " C12 ", s57\n\t"                               \
  "v_perm_b32 v35, " C15 ", " C14 ", s58\n\t"                               \
  "v_or_b32 v39, v34, v35\n\t"

// set-up of the 5-8-row tile: constants, the first ring loads (ONE_MORE: a third,
// into slot C), zeroed accumulators, row / group counters
#define ECW2_TILE_INIT(MODE, ONE_MORE)                                            \
  "v_mov_b32 v40, %[col]\n\t"                                               \
  "v_mov_b32 v33, 0xf0f0f0f0\n\t"                                           \
  "v_mov_b32 v41, 0xff\n\t"                                                 \
  "s_mov_b32 s50, 0x0c0c0400\n\t"                                           \
  "s_mov_b32 s51, 0x0c0c0401\n\t"                                           \
  "s_mov_b32 s52, 0x0c0c0402\n\t"                                           \
  "s_mov_b32 s53, 0x0c0c0403\n\t"                                           \
  ECW_ROWPTR_INIT_##MODE                                                    \
  ECW_LOAD_A ECW_NEXTROW_##MODE "s_waitcnt lgkmcnt(0)\n\t"                  \
  ECW_LOAD_B ECW_NEXTROW_##MODE                                             \
  ONE_MORE                                                                  \
  "v_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\tv_mov_b32 v15, 0\n\t" \
  "v_mov_b32 v16, 0\n\tv_mov_b32 v17, 0\n\tv_mov_b32 v18, 0\n\tv_mov_b32 v19, 0\n\t" \
  "v_mov_b32 v20, 0\n\tv_mov_b32 v21, 0\n\tv_mov_b32 v22, 0\n\tv_mov_b32 v23, 0\n\t" \
  "v_mov_b32 v24, 0\n\tv_mov_b32 v25, 0\n\tv_mov_b32 v26, 0\n\tv_mov_b32 v27, 0\n\t" \
  "v_mov_b32 v74, 0\n\tv_mov_b32 v75, 0\n\tv_mov_b32 v76, 0\n\tv_mov_b32 v77, 0\n\t" \
  "v_mov_b32 v78, 0\n\tv_mov_b32 v79, 0\n\tv_mov_b32 v80, 0\n\tv_mov_b32 v81, 0\n\t" \
  "v_mov_b32 v82, 0\n\tv_mov_b32 v83, 0\n\tv_mov_b32 v84, 0\n\tv_mov_b32 v85, 0\n\t" \
  "v_mov_b32 v86, 0\n\tv_mov_b32 v87, 0\n\tv_mov_b32 v88, 0\n\tv_mov_b32 v89, 0\n\t" \
  "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\tv_mov_b32 v30, 0\n\tv_mov_b32 v31, 0\n\t" \
  ECW2_ROW_YZERO                                                            \
  "s_mov_b32 s44, 0\n\t"                                                    \
  "s_mov_b32 s59, 0\n\t"                                                    \
  "s_mov_b32 s46, %[lds]\n\t"                                               \
  ECW_LPTR_INIT_##MODE                                                      \
  "s_min_u32 s45, %[r], %[k]\n\t"                                           \

// global rows l: byte (l & 3) of bank l >> 2 -> output row l (v[36:39])
#define ECW2_GLOBAL_ROWS(MODE)                                                    \
  ECW_GPTR_INIT_##MODE                                                      \
  "s_mov_b32 s56, 0\n\t"                                                    \
  "30:\n\t"                                                                 \
  "s_cmp_ge_u32 s56, %[nrows]\n\t"                                          \
  "s_cbranch_scc1 31f\n\t"                                                  \
  "s_and_b32 s49, s56, 3\n\t"                                               \
  "s_add_u32 s57, s49, 4\n\t"                                               \
  "s_lshl_b32 s58, s57, 24\n\t"                                             \
  "s_lshl_b32 s57, s57, 8\n\t"                                              \
  "s_or_b32 s57, s57, s49\n\t"                                              \
  "s_or_b32 s57, s57, 0x0c0c0000\n\t"                                       \
  "s_lshl_b32 s49, s49, 16\n\t"                                             \
  "s_or_b32 s58, s58, s49\n\t"                                              \
  "s_or_b32 s58, s58, 0x0c0c\n\t"                                           \
  "s_cmp_ge_u32 s56, 4\n\t"                                                 \
  "s_cbranch_scc1 32f\n\t"                                                  \
  ECW2_TRANSPOSE("v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19",    \
                 "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27")    \
  "s_branch 33f\n\t"                                                        \
  "32:\n\t"                                                                 \
  ECW2_TRANSPOSE("v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",    \
                 "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89")    \
  "33:\n\t"                                                                 \
  ECW_GPTR_GET_##MODE                                                       \
  ECW_ASM_GSTORE("v[36:39]", "s[54:55]")                                    \
  "s_nop 1\n\t"                                                             \
  ECW_GPTR_NEXT_##MODE                                                      \
  "s_add_u32 s56, s56, 1\n\t"                                               \
  "s_branch 30b\n\t"                                                        \
  "31:"

#define ECW2_TILE_ASM(BND, XL, END, MODE)                                          \
  ECW2_TILE_INIT(MODE, )                                                    \
  "10:\n\t"                                                                 \
  "s_add_u32 s49, s44, 3\n\t"                                               \
  "s_cmp_ge_u32 s49, %[k]\n\t"                                              \
  "s_cbranch_scc1 11f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW2_STEP_##MODE(ECW2_ROW_PRE_A(XL), ECW_LOAD_A, ECW_NEXTROW_##MODE, BND) \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW2_STEP_##MODE(ECW2_ROW_PRE_B(XL), ECW_LOAD_B, ECW_NEXTROW_##MODE, BND) \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_branch 10b\n\t"                                                        \
  "11:\n\t"                                                                 \
  "s_sub_u32 s49, %[k], s44\n\t"                                            \
  "s_cmp_eq_u32 s49, 3\n\t"                                                 \
  "s_cbranch_scc0 12f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW2_STEP_##MODE(ECW2_ROW_PRE_A(XL), ECW_LOAD_A, , BND)                   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW2_ROW_B(XL) BND                                                        \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW2_ROW_A(XL) BND                                                        \
  "s_branch 13f\n\t"                                                        \
  "12:\n\t"                                                                 \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW2_ROW_A(XL) BND                                                        \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW2_ROW_B(XL) BND                                                        \
  "13:\n\t"                                                                 \
  ECW2_ROW_DRAIN                                                            \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW2_GLOBAL_ROWS(MODE)

// the three-slot ring of the 5-8-row tile (slot C = v[36:39], as ECW_TILE_ASM3)
#define ECW2_ROW_C(XL) ECW2_ROW("v36", "v37", "v38", "v39", XL)
#define ECW2_ROW_PRE_C(XL) ECW2_ROW_PRE("v36", "v37", "v38", "v39", XL)
#define ECW2_TILE_ASM3(BND, XL, END, MODE)                                         \
  ECW2_TILE_INIT(MODE, "s_waitcnt lgkmcnt(0)\n\t" ECW_LOAD_C ECW_NEXTROW_##MODE) \
  ECW_RING3_ROWS(ECW2, BND, XL, MODE)                                       \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW2_GLOBAL_ROWS(MODE)

#define ECW2_TILE_OPERANDS                                                          \
  ECW_TILE_OPERANDS, "s63", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67",  \
    "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80",      \
    "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89"
#define ECW2_TILE_OPERANDS_PARK                                                     \
  ECW2_TILE_OPERANDS, "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99",       \
    "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109"

// ---------------------------------------------------------------------------
// 9-16 global rows (NW = 4): one 16-byte table entry per nibble (rows 4e..4e+3
// in dword e; records of 512 B, lo-nibble entries at +0, hi at +256, so a
// record's low byte is that of the table base), looked up with ds_read_b128
// (4 LDS cycles, conflict-free: a lookup's 16 entries cover the 64 banks), and
// four banks of 16 packed accumulators. One pass over the data instead of two
// passes of <= 8 rows. The tables reach past 64 KiB for k > 128, so the record
// address enters the lookup address with two bytes (selectors 0x0C0504xx).
// Lookups go in sets of four (two data bytes, lo and hi): set X v[42:57], set Y
// v[58:73], each tuple's address in its first register; nibble words v34/v35
// (nibble * 16: lo = (W << 4) & 0xF0.., hi = W & 0xF0..), v33 = 0xF0F0F0F0.
// Accumulators: rows 0-3 v[12:27], 4-7 v[74:89], 8-11 v[90:105], 12-15
// v[106:121] (byte column c of the lane's 16 in the c-th register of each
// bank); parked local parities v[122:141]. Rows are software-pipelined: the
// last Y set of a row is folded after the next row's first X set is issued.
#define ECW4_NIB(W)                                  \
  "v_lshlrev_b32 v34, 4, " W "\n\t"                  \
  "v_and_or_b32 v34, v34, v33, s48\n\t"              \
  "v_and_or_b32 v35, " W ", v33, s48\n\t"
// lookup addresses of two data bytes (selectors SA, SB) of the nibble words
#define ECW4_ADDR(SA, SB, A0, A1, A2, A3)            \
  "v_perm_b32 " A0 ", v32, v34, " SA "\n\t"          \
  "v_perm_b32 " A1 ", v32, v35, " SA "\n\t"          \
  "v_perm_b32 " A2 ", v32, v34, " SB "\n\t"          \
  "v_perm_b32 " A3 ", v32, v35, " SB "\n\t"
#define ECW4_ADDR_X01 ECW4_ADDR("s50", "s51", "v42", "v46", "v50", "v54")
#define ECW4_ADDR_Y23 ECW4_ADDR("s52", "s53", "v58", "v62", "v66", "v70")
#define ECW4_READ_X                                  \
  "ds_read_b128 v[42:45], v42\n\t"                   \
  "ds_read_b128 v[46:49], v46 offset:256\n\t"        \
  "ds_read_b128 v[50:53], v50\n\t"                   \
  "ds_read_b128 v[54:57], v54 offset:256\n\t"
#define ECW4_READ_Y                                  \
  "ds_read_b128 v[58:61], v58\n\t"                   \
  "ds_read_b128 v[62:65], v62 offset:256\n\t"        \
  "ds_read_b128 v[66:69], v66\n\t"                   \
  "ds_read_b128 v[70:73], v70 offset:256\n\t"
// byte column p: lo entry (L0..L3) ^ hi entry (H0..H3) into the four banks
#define ECW4_FOLD1(C, D, E, F, L0, L1, L2, L3, H0, H1, H2, H3)     \
  "v_bitop3_b32 " C ", " C ", " L0 ", " H0 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " D ", " D ", " L1 ", " H1 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " E ", " E ", " L2 ", " H2 " bitop3:0x96\n\t"      \
  "v_bitop3_b32 " F ", " F ", " L3 ", " H3 " bitop3:0x96\n\t"
// byte columns p and p + 1 from set X / set Y (P = p, Q = p + 1 as numbers)
#define ECW4_FOLD_X(P, Q)                                                                           \
  ECW4_FOLD1("v" #P, "v" ECW4_D(P), "v" ECW4_E(P), "v" ECW4_F(P), "v42", "v43", "v44", "v45", "v46", \
             "v47", "v48", "v49")                                                                   \
  ECW4_FOLD1("v" #Q, "v" ECW4_D(Q), "v" ECW4_E(Q), "v" ECW4_F(Q), "v50", "v51", "v52", "v53", "v54", \
             "v55", "v56", "v57")
#define ECW4_FOLD_Y(P, Q)                                                                           \
  ECW4_FOLD1("v" #P, "v" ECW4_D(P), "v" ECW4_E(P), "v" ECW4_F(P), "v58", "v59", "v60", "v61", "v62", \
             "v63", "v64", "v65")                                                                   \
  ECW4_FOLD1("v" #Q, "v" ECW4_D(Q), "v" ECW4_E(Q), "v" ECW4_F(Q), "v66", "v67", "v68", "v69", "v70", \
             "v71", "v72", "v73")
// bank registers of byte column c (bank C: v12 + c): D = v74 + c, E = v90 + c,
// F = v106 + c, spelled out (P is the bank-C register number 12..27)
#define ECW4_D(P) ECW4_D_##P
#define ECW4_E(P) ECW4_E_##P
#define ECW4_F(P) ECW4_F_##P
#define ECW4_D_12 "74"
#define ECW4_D_13 "75"
#define ECW4_D_14 "76"
#define ECW4_D_15 "77"
#define ECW4_D_16 "78"
#define ECW4_D_17 "79"
#define ECW4_D_18 "80"
#define ECW4_D_19 "81"
#define ECW4_D_20 "82"
#define ECW4_D_21 "83"
#define ECW4_D_22 "84"
#define ECW4_D_23 "85"
#define ECW4_D_24 "86"
#define ECW4_D_25 "87"
#define ECW4_D_26 "88"
#define ECW4_D_27 "89"
#define ECW4_E_12 "90"
#define ECW4_E_13 "91"
#define ECW4_E_14 "92"
#define ECW4_E_15 "93"
#define ECW4_E_16 "94"
#define ECW4_E_17 "95"
#define ECW4_E_18 "96"
#define ECW4_E_19 "97"
#define ECW4_E_20 "98"
#define ECW4_E_21 "99"
#define ECW4_E_22 "100"
#define ECW4_E_23 "101"
#define ECW4_E_24 "102"
#define ECW4_E_25 "103"
#define ECW4_E_26 "104"
#define ECW4_E_27 "105"
#define ECW4_F_12 "106"
#define ECW4_F_13 "107"
#define ECW4_F_14 "108"
#define ECW4_F_15 "109"
#define ECW4_F_16 "110"
#define ECW4_F_17 "111"
#define ECW4_F_18 "112"
#define ECW4_F_19 "113"
#define ECW4_F_20 "114"
#define ECW4_F_21 "115"
#define ECW4_F_22 "116"
#define ECW4_F_23 "117"
#define ECW4_F_24 "118"
#define ECW4_F_25 "119"
#define ECW4_F_26 "120"
#define ECW4_F_27 "121"
// One data row from ring slot R0..R3 (s46 = its LDS table record). PRE ends
// where the slot's registers are last read; the previous row's last Y set
// (byte columns 14, 15) is folded after this row's first X set is issued.
#define ECW4_ROW_PRE(R0, R1, R2, R3, XL)           \
  "s_lshr_b32 s47, s46, 8\n\t"                     \
  "s_and_b32 s48, s46, 0xff\n\t"                   \
  "s_mul_i32 s48, s48, 0x01010101\n\t"             \
  "v_mov_b32 v32, s47\n\t"                         \
  ECW4_NIB(R0) ECW4_ADDR_X01 ECW4_READ_X           \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_Y(26, 27)                              \
  ECW4_ADDR_Y23 ECW4_READ_Y                        \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_X(12, 13)                              \
  ECW4_NIB(R1) ECW4_ADDR_X01 ECW4_READ_X           \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_Y(14, 15)                              \
  ECW4_ADDR_Y23 ECW4_READ_Y                        \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_X(16, 17)                              \
  ECW4_NIB(R2) ECW4_ADDR_X01 ECW4_READ_X           \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_Y(18, 19)                              \
  ECW4_ADDR_Y23 ECW4_READ_Y                        \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_X(20, 21)                              \
  ECW4_NIB(R3) ECW4_ADDR_X01 ECW4_READ_X           \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_Y(22, 23)                              \
  ECW4_ADDR_Y23 ECW4_READ_Y                        \
  ECW_LACC_##XL(R0, R1, R2, R3)                    \
  "s_add_u32 s46, s46, 512\n\t"
#define ECW4_ROW_POST                              \
  "s_waitcnt lgkmcnt(4)\n\t"                       \
  ECW4_FOLD_X(24, 25)
#define ECW4_ROW_DRAIN "s_waitcnt lgkmcnt(0)\n\t" ECW4_FOLD_Y(26, 27)
#define ECW4_ROW_YZERO                                                                   \
  "v_mov_b32 v58, 0\n\tv_mov_b32 v59, 0\n\tv_mov_b32 v60, 0\n\tv_mov_b32 v61, 0\n\t"     \
  "v_mov_b32 v62, 0\n\tv_mov_b32 v63, 0\n\tv_mov_b32 v64, 0\n\tv_mov_b32 v65, 0\n\t"     \
  "v_mov_b32 v66, 0\n\tv_mov_b32 v67, 0\n\tv_mov_b32 v68, 0\n\tv_mov_b32 v69, 0\n\t"     \
  "v_mov_b32 v70, 0\n\tv_mov_b32 v71, 0\n\tv_mov_b32 v72, 0\n\tv_mov_b32 v73, 0\n\t"
#define ECW4_ROW(R0, R1, R2, R3, XL) ECW4_ROW_PRE(R0, R1, R2, R3, XL) ECW4_ROW_POST
#define ECW4_ROW_A(XL) ECW4_ROW("v4", "v5", "v6", "v7", XL)
#define ECW4_ROW_B(XL) ECW4_ROW("v8", "v9", "v10", "v11", XL)
#define ECW4_ROW_PRE_A(XL) ECW4_ROW_PRE("v4", "v5", "v6", "v7", XL)
#define ECW4_ROW_PRE_B(XL) ECW4_ROW_PRE("v8", "v9", "v10", "v11", XL)
#define ECW4_STEP_SLAB(PRE, LOAD, NEXT, BND) PRE LOAD NEXT ECW4_ROW_POST BND
#define ECW4_STEP_TAB(PRE, LOAD, NEXT, BND) PRE ECW4_ROW_POST BND ECW_LDWAIT_TAB LOAD NEXT

#define ECW4_BOUNDARY_PARK                                  \
  "s_add_u32 s49, s44, 1\n\t"                               \
  "s_cmp_eq_u32 s49, s45\n\t"                               \
  "s_cbranch_scc0 20f\n\t"                                  \
  ECW_PARK(0, "v122", "v123", "v124", "v125", 21)           \
  ECW_PARK(1, "v126", "v127", "v128", "v129", 22)           \
  ECW_PARK(2, "v130", "v131", "v132", "v133", 23)           \
  ECW_PARK(3, "v134", "v135", "v136", "v137", 24)           \
  ECW_PARK(4, "v138", "v139", "v140", "v141", 25)           \
  "26:\n\t"                                                 \
  "s_add_u32 s59, s59, 1\n\t"                               \
  "s_add_u32 s45, s45, %[r]\n\t"                            \
  "s_min_u32 s45, s45, %[k]\n\t"                            \
  ECW_LRESET_1                                              \
  "20:\n\t"
#define ECW4_STORE_PARKED(MODE)                                             \
  ECW_LPTR_INIT_##MODE                                                      \
  ECW_UNPARK(0, "v[122:125]", MODE) ECW_UNPARK(1, "v[126:129]", MODE)       \
  ECW_UNPARK(2, "v[130:133]", MODE) ECW_UNPARK(3, "v[134:137]", MODE)       \
  ECW_UNPARK(4, "v[138:141]", MODE)                                         \
  "27:\n\t"

// set-up of the 9-16-row tile (ONE_MORE: a third ring load, into slot C)
#define ECW4_TILE_INIT(MODE, ONE_MORE)                                            \
  "v_mov_b32 v40, %[col]\n\t"                                               \
  "v_mov_b32 v33, 0xf0f0f0f0\n\t"                                           \
  "s_mov_b32 s50, 0x0c050400\n\t"                                           \
  "s_mov_b32 s51, 0x0c050401\n\t"                                           \
  "s_mov_b32 s52, 0x0c050402\n\t"                                           \
  "s_mov_b32 s53, 0x0c050403\n\t"                                           \
  ECW_ROWPTR_INIT_##MODE                                                    \
  ECW_LOAD_A ECW_NEXTROW_##MODE "s_waitcnt lgkmcnt(0)\n\t"                  \
  ECW_LOAD_B ECW_NEXTROW_##MODE                                             \
  ONE_MORE                                                                  \
  "v_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\tv_mov_b32 v15, 0\n\t" \
  "v_mov_b32 v16, 0\n\tv_mov_b32 v17, 0\n\tv_mov_b32 v18, 0\n\tv_mov_b32 v19, 0\n\t" \
  "v_mov_b32 v20, 0\n\tv_mov_b32 v21, 0\n\tv_mov_b32 v22, 0\n\tv_mov_b32 v23, 0\n\t" \
  "v_mov_b32 v24, 0\n\tv_mov_b32 v25, 0\n\tv_mov_b32 v26, 0\n\tv_mov_b32 v27, 0\n\t" \
  "v_mov_b32 v74, 0\n\tv_mov_b32 v75, 0\n\tv_mov_b32 v76, 0\n\tv_mov_b32 v77, 0\n\t" \
  "v_mov_b32 v78, 0\n\tv_mov_b32 v79, 0\n\tv_mov_b32 v80, 0\n\tv_mov_b32 v81, 0\n\t" \
  "v_mov_b32 v82, 0\n\tv_mov_b32 v83, 0\n\tv_mov_b32 v84, 0\n\tv_mov_b32 v85, 0\n\t" \
  "v_mov_b32 v86, 0\n\tv_mov_b32 v87, 0\n\tv_mov_b32 v88, 0\n\tv_mov_b32 v89, 0\n\t" \
  "v_mov_b32 v90, 0\n\tv_mov_b32 v91, 0\n\tv_mov_b32 v92, 0\n\tv_mov_b32 v93, 0\n\t" \
  "v_mov_b32 v94, 0\n\tv_mov_b32 v95, 0\n\tv_mov_b32 v96, 0\n\tv_mov_b32 v97, 0\n\t" \
  "v_mov_b32 v98, 0\n\tv_mov_b32 v99, 0\n\tv_mov_b32 v100, 0\n\tv_mov_b32 v101, 0\n\t" \
  "v_mov_b32 v102, 0\n\tv_mov_b32 v103, 0\n\tv_mov_b32 v104, 0\n\tv_mov_b32 v105, 0\n\t" \
  "v_mov_b32 v106, 0\n\tv_mov_b32 v107, 0\n\tv_mov_b32 v108, 0\n\tv_mov_b32 v109, 0\n\t" \
  "v_mov_b32 v110, 0\n\tv_mov_b32 v111, 0\n\tv_mov_b32 v112, 0\n\tv_mov_b32 v113, 0\n\t" \
  "v_mov_b32 v114, 0\n\tv_mov_b32 v115, 0\n\tv_mov_b32 v116, 0\n\tv_mov_b32 v117, 0\n\t" \
  "v_mov_b32 v118, 0\n\tv_mov_b32 v119, 0\n\tv_mov_b32 v120, 0\n\tv_mov_b32 v121, 0\n\t" \
  "v_mov_b32 v28, 0\n\tv_mov_b32 v29, 0\n\tv_mov_b32 v30, 0\n\tv_mov_b32 v31, 0\n\t" \
  ECW4_ROW_YZERO                                                            \
  "s_mov_b32 s44, 0\n\t"                                                    \
  "s_mov_b32 s59, 0\n\t"                                                    \
  "s_mov_b32 s46, %[lds]\n\t"                                               \
  ECW_LPTR_INIT_##MODE                                                      \
  "s_min_u32 s45, %[r], %[k]\n\t"                                           \

// global rows l: byte (l & 3) of bank l >> 2 -> output row l (v[36:39])
#define ECW4_GLOBAL_ROWS(MODE)                                                    \
  ECW_GPTR_INIT_##MODE                                                      \
  "s_mov_b32 s56, 0\n\t"                                                    \
  "30:\n\t"                                                                 \
  "s_cmp_ge_u32 s56, %[nrows]\n\t"                                          \
  "s_cbranch_scc1 31f\n\t"                                                  \
  "s_and_b32 s49, s56, 3\n\t"                                               \
  "s_add_u32 s57, s49, 4\n\t"                                               \
  "s_lshl_b32 s58, s57, 24\n\t"                                             \
  "s_lshl_b32 s57, s57, 8\n\t"                                              \
  "s_or_b32 s57, s57, s49\n\t"                                              \
  "s_or_b32 s57, s57, 0x0c0c0000\n\t"                                       \
  "s_lshl_b32 s49, s49, 16\n\t"                                             \
  "s_or_b32 s58, s58, s49\n\t"                                              \
  "s_or_b32 s58, s58, 0x0c0c\n\t"                                           \
  "s_cmp_ge_u32 s56, 8\n\t"                                                 \
  "s_cbranch_scc1 36f\n\t"                                                  \
  "s_cmp_ge_u32 s56, 4\n\t"                                                 \
  "s_cbranch_scc1 32f\n\t"                                                  \
  ECW2_TRANSPOSE("v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19",    \
                 "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27")    \
  "s_branch 33f\n\t"                                                        \
  "32:\n\t"                                                                 \
  ECW2_TRANSPOSE("v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",    \
                 "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89")    \
  "s_branch 33f\n\t"                                                        \
  "36:\n\t"                                                                 \
  "s_cmp_ge_u32 s56, 12\n\t"                                                \
  "s_cbranch_scc1 37f\n\t"                                                  \
  ECW2_TRANSPOSE("v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97",    \
                 "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105") \
  "s_branch 33f\n\t"                                                        \
  "37:\n\t"                                                                 \
  ECW2_TRANSPOSE("v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", \
                 "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121") \
  "33:\n\t"                                                                 \
  ECW_GPTR_GET_##MODE                                                       \
  ECW_ASM_GSTORE("v[36:39]", "s[54:55]")                                    \
  "s_nop 1\n\t"                                                             \
  ECW_GPTR_NEXT_##MODE                                                      \
  "s_add_u32 s56, s56, 1\n\t"                                               \
  "s_branch 30b\n\t"                                                        \
  "31:"

#define ECW4_TILE_ASM(BND, XL, END, MODE)                                          \
  ECW4_TILE_INIT(MODE, )                                                    \
  "10:\n\t"                                                                 \
  "s_add_u32 s49, s44, 3\n\t"                                               \
  "s_cmp_ge_u32 s49, %[k]\n\t"                                              \
  "s_cbranch_scc1 11f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW4_STEP_##MODE(ECW4_ROW_PRE_A(XL), ECW_LOAD_A, ECW_NEXTROW_##MODE, BND) \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW4_STEP_##MODE(ECW4_ROW_PRE_B(XL), ECW_LOAD_B, ECW_NEXTROW_##MODE, BND) \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_branch 10b\n\t"                                                        \
  "11:\n\t"                                                                 \
  "s_sub_u32 s49, %[k], s44\n\t"                                            \
  "s_cmp_eq_u32 s49, 3\n\t"                                                 \
  "s_cbranch_scc0 12f\n\t"                                                  \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW4_STEP_##MODE(ECW4_ROW_PRE_A(XL), ECW_LOAD_A, , BND)                   \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW4_ROW_B(XL) BND                                                        \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW4_ROW_A(XL) BND                                                        \
  "s_branch 13f\n\t"                                                        \
  "12:\n\t"                                                                 \
  "s_waitcnt vmcnt(1)\n\t"                                                  \
  ECW4_ROW_A(XL) BND                                                        \
  "s_add_u32 s44, s44, 1\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"                                                  \
  ECW4_ROW_B(XL) BND                                                        \
  "13:\n\t"                                                                 \
  ECW4_ROW_DRAIN                                                            \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW4_GLOBAL_ROWS(MODE)

#define ECW4_ROW_C(XL) ECW4_ROW("v36", "v37", "v38", "v39", XL)
#define ECW4_ROW_PRE_C(XL) ECW4_ROW_PRE("v36", "v37", "v38", "v39", XL)
#define ECW4_TILE_ASM3(BND, XL, END, MODE)                                         \
  ECW4_TILE_INIT(MODE, "s_waitcnt lgkmcnt(0)\n\t" ECW_LOAD_C ECW_NEXTROW_##MODE) \
  ECW_RING3_ROWS(ECW4, BND, XL, MODE)                                       \
  ECW_WRITE_WINDOW                                                          \
  END                                                                       \
  ECW4_GLOBAL_ROWS(MODE)

#define ECW4_TILE_OPERANDS                                                          \
  ECW2_TILE_OPERANDS, "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99",        \
    "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", \
    "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121"
#define ECW4_TILE_OPERANDS_PARK                                                     \
  ECW4_TILE_OPERANDS, "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130",     \
    "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141"

namespace ecw {
namespace {

// LOCAL: kLocalNone / kLocalXor / kLocalZero (ecw_internal.hpp); PARK: keep
// the (<= 5) local parities in registers until the end of the tile (literal
// mode always stores its zero L blocks there); TAB:
// block pointers come from pointer tables (see ECW_ROWPTR_INIT_TAB). Requires
// k >= 2, a full tile (every lane's 16 bytes in range) and exec = all lanes.
#define ECW_TILE_CALL(TILE, MODE)                                                           \
  if constexpr (LOCAL == kLocalNone) {                                                   \
    asm volatile(TILE(ECW_BOUNDARY_NONE, 0, , MODE) ECW_TILE_OPERANDS);           \
  } else if constexpr (LOCAL == kLocalXor && PARK) {                                     \
    asm volatile(TILE(ECW_BOUNDARY_PARK, 1, ECW_STORE_PARKED(MODE), MODE)        \
                     ECW_TILE_OPERANDS_PARK);                                            \
  } else if constexpr (LOCAL == kLocalXor) {                                             \
    asm volatile(TILE(ECW_BOUNDARY(1, MODE), 1, , MODE) ECW_TILE_OPERANDS);       \
  } else {                                                                               \
    asm volatile(TILE(ECW_BOUNDARY_COUNT, 0, ECW_STORE_ZEROS(MODE), MODE)          \
                     ECW_TILE_OPERANDS);                                                 \
  }

#define ECW2_TILE_CALL(TILE, MODE)                                                           \
  if constexpr (LOCAL == kLocalNone) {                                                   \
    asm volatile(TILE(ECW_BOUNDARY_NONE, 0, , MODE) ECW2_TILE_OPERANDS);         \
  } else if constexpr (LOCAL == kLocalXor && PARK) {                                     \
    asm volatile(TILE(ECW2_BOUNDARY_PARK, 1, ECW2_STORE_PARKED(MODE), MODE)     \
                     ECW2_TILE_OPERANDS_PARK);                                           \
  } else if constexpr (LOCAL == kLocalXor) {                                             \
    asm volatile(TILE(ECW_BOUNDARY(1, MODE), 1, , MODE) ECW2_TILE_OPERANDS);     \
  } else {                                                                               \
    asm volatile(TILE(ECW_BOUNDARY_COUNT, 0, ECW_STORE_ZEROS(MODE), MODE)         \
                     ECW2_TILE_OPERANDS);                                                \
  }

#define ECW4_TILE_CALL(TILE, MODE)                                                           \
  if constexpr (LOCAL == kLocalNone) {                                                   \
    asm volatile(TILE(ECW_BOUNDARY_NONE, 0, , MODE) ECW4_TILE_OPERANDS);         \
  } else if constexpr (LOCAL == kLocalXor && PARK) {                                     \
    asm volatile(TILE(ECW4_BOUNDARY_PARK, 1, ECW4_STORE_PARKED(MODE), MODE)     \
                     ECW4_TILE_OPERANDS_PARK);                                           \
  } else if constexpr (LOCAL == kLocalXor) {                                             \
    asm volatile(TILE(ECW_BOUNDARY(1, MODE), 1, , MODE) ECW4_TILE_OPERANDS);     \
  } else {                                                                               \
    asm volatile(TILE(ECW_BOUNDARY_COUNT, 0, ECW_STORE_ZEROS(MODE), MODE)         \
                     ECW4_TILE_OPERANDS);                                                \
  }

// NW = 1: <= 4 global rows (u32 table entries); NW = 2: 5-8 rows (u64
// entries); NW = 4: 9-16 rows (16-byte entries)
template <int LOCAL, bool PARK, bool TAB, int NW = 1>
__device__ __forceinline__ void encode_tile_asm(const uint8_t* row0, uint8_t* lrow0, uint8_t* grow0, uint64_t bstride,
                                                uint64_t pbstride, int k, int r, int nrows, uint32_t lds,
                                                uint32_t col, uint32_t wmask, uint32_t ww) {
  const uint32_t bslo = static_cast<uint32_t>(bstride), bshi = static_cast<uint32_t>(bstride >> 32);
  const uint32_t pbslo = static_cast<uint32_t>(pbstride), pbshi = static_cast<uint32_t>(pbstride >> 32);
  const bool ring3 = k >= 3 && (kAsmRing3 == 2 || (kAsmRing3 == 1 && ww != 0));  // uniform: a scalar branch
  const bool ring3_nw2 = k >= 3 && kAsmRing3Nw2 != 0;
  const bool ring3_nw4 = k >= 3 && kAsmRing3Nw4 != 0;
  if constexpr (NW == 4) {
    if constexpr (TAB) {
      if (ring3_nw4) {
        ECW4_TILE_CALL(ECW4_TILE_ASM3, TAB)
      } else {
        ECW4_TILE_CALL(ECW4_TILE_ASM, TAB)
      }
    } else {
      if (ring3_nw4) {
        ECW4_TILE_CALL(ECW4_TILE_ASM3, SLAB)
      } else {
        ECW4_TILE_CALL(ECW4_TILE_ASM, SLAB)
      }
    }
  } else if constexpr (NW == 2) {
    if constexpr (TAB) {
      if (ring3_nw2) {
        ECW2_TILE_CALL(ECW2_TILE_ASM3, TAB)
      } else {
        ECW2_TILE_CALL(ECW2_TILE_ASM, TAB)
      }
    } else {
      if (ring3_nw2) {
        ECW2_TILE_CALL(ECW2_TILE_ASM3, SLAB)
      } else {
        ECW2_TILE_CALL(ECW2_TILE_ASM, SLAB)
      }
    }
  } else if constexpr (TAB) {
    if (ring3) {
      ECW_TILE_CALL(ECW_TILE_ASM3, TAB)
    } else {
      ECW_TILE_CALL(ECW_TILE_ASM, TAB)
    }
  } else {
    if (ring3) {
      ECW_TILE_CALL(ECW_TILE_ASM3, SLAB)
    } else {
      ECW_TILE_CALL(ECW_TILE_ASM, SLAB)
    }
  }
}

}  // namespace
}  // namespace ecw
