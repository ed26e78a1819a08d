/* Measurement-only ceiling modes of the A/B build (libcallfs_rs_ab.so, built on demand by
 * `python callfs_amd/build.py --ab` into build/ab/ and loaded by the development tools
 * through CALLFS_RS_LIB). The product library (include/callfs_rs.h) implements only
 * RS_CEIL_READ and RS_CEIL_WRITE and returns RS_E_ARG for these. */
#ifndef CALLFS_RS_AB_H
#define CALLFS_RS_AB_H

#include "../include/callfs_rs.h"

/* the production kernel's no-lookup form: the same loads, stores and table prologue, one XOR
 * per input dword in place of the lookups (junk in the written shards; may flag status) */
#define RS_CEIL_NOLOOKUP 0
/* the write streams alone from each row's first 64 / 128 / 256-B boundary on (every wave's
 * 1 KiB store aligned to that; consecutive tiles) */
#define RS_CEIL_WRITE_AL64 3
#define RS_CEIL_WRITE_AL128 4
#define RS_CEIL_WRITE_AL256 5
/* the read streams alone from each shard's first 64 / 128 / 256-B boundary on */
#define RS_CEIL_READ_AL64 6
#define RS_CEIL_READ_AL128 7
#define RS_CEIL_READ_AL256 8

#endif
