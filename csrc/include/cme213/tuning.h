// Process-wide tuning knobs of the native library (arm selection, chunk
// heights, spin bounds, rehearsal delays) -- ONE table, read per call.
//
// Every knob starts from its CME_* environment variable (or the measured
// default) the first time it is read, and can be changed at run time through
// cme_tune_set / cme_tune_reset (Python: cme213x.utils.tuning), so a test or
// a sweep selects an arm in-process instead of spawning a subprocess with a
// different environment. Launchers read the knob on every call (one relaxed
// atomic load); nothing caches it in a function-local static.
#pragma once

namespace cme {

enum TuneKey : int {
    kTunePipeVW = 0,       // CME_PIPE_VW: 0 measured default (8 columns per lane at order 8), 4 / 8 forced
    kTunePipeChunk,        // CME_PIPE_CHUNK: rows per pipelined-pass task (0 = rule)
    kTunePipePerCU,        // CME_PIPE_PER_CU: task target per CU (0 = rule)
    kTunePipeThinMin,      // CME_PIPE_THIN_MIN: minimum chunk of thin (border) regions
    kTuneDistSchedule,     // CME_DIST_SCHEDULE: 2 fused (default), 0 events, 1 one stream
    kTuneDistEventScope,   // CME_DIST_EVENT_SCOPE: 0 system-scope events, 1 device-scope
    kTuneDistVerbose,      // CME_DIST_VERBOSE: log the queue probe
    kTuneDistGateSpins,    // CME_DIST_GATE_SPINS: polls of a fused border wait before it gives up
    kTuneDistFakeXchgUs,   // CME_DIST_FAKE_XCHG_US: rehearsal / test delay of each exchange
    kTuneRadixMaxBlocks,   // CME_RADIX_MAXBLOCKS: reduce-then-scan grid cap
    kTuneRadixDS,          // CME_RADIX_DS: downsweep arm bits (1 group atomics, 2 prefetch, 4 8192-key tiles, 8 lane ranks, 16 16384-key tiles with lane ranks)
    kTuneStream2Chunk,     // CME_STREAM2_CHUNK
    kTuneStreamNChunk,     // CME_STREAMN_CHUNK
    kTuneStreamNRounds,    // CME_STREAMN_ROUNDS
    kTuneStreamNMinChunk,  // CME_STREAMN_MINCHUNK
    kTuneStreamNThinWaves, // CME_STREAMN_THIN_WAVES
    kTuneStreamNCapPct,    // CME_STREAMN_CAPPCT
    kTuneSpmvScanMulti,    // CME_SPMVSCAN_MULTI
    kTuneSpmvNT,           // CME_SPMV_NT: aligned-CSR stream loads (0 plain, 1 non-temporal, 2 by size)
    kTuneSpmvDia1,         // CME_SPMV_DIA1
    kTunePipeTaper,        // CME_PIPE_TAPER: half-height last chunks per strip of a multi-round pass (0 off, -1 auto)
    kTuneRadixUpUnr,       // CME_RADIX_UP_UNR: radix upsweep 16-B loads in flight per lane (4, 8, 16)
    kTuneRadixOsLanes,     // CME_RADIX_OS_LANES: onesweep ranks, 1 lane order where the probe passed, 0 ballot match
    kTuneFlowPerCU,        // CME_FLOW_PER_CU: task target per CU of the dataflow launch (0 = the pipelined pass's rule)
    kTuneFlowSpins,        // CME_FLOW_SPINS: polls of a dataflow dependency wait before it gives up
    kTuneFlowMode,         // CME_FLOW_MODE: diagnostics of the dataflow hand-off (fence scopes)
    kTuneSpmvStreamRows,   // CME_SPMV_STREAM_ROWS: CSR-stream rows per block (0 = by mean row length)
    kTuneTileResMinR,      // CME_TILE_RES_MINR: rows per band at least in the resident tiles' steps
    kTuneSpmvShortRpt,     // CME_SPMV_SHORT_RPT: CSR-short rows per lane (1, 2, 4)
    kTuneMergePart,        // CME_MERGE_PART: merge sort partitions: 4 / 8 / 16 / 32 / 64 lanes per tile in one search launch per pass (other positive: 64), 0 in-block searches, -1 auto (8 from 8M keys)
    kTuneMergeTile,        // CME_MERGE_TILE: merge sort output tile per merge-pass block, 4096 or 8192 keys (8192 with partitions)
    kTuneMergeBlock,       // CME_MERGE_BLOCK: merge sort block-sort tile, 8192 (512 lanes) or 16384 keys (1024 lanes); 0 auto (16384 for keys only from 4M)
    kTuneMergeSamples,     // CME_MERGE_SAMPLES: merge sort run samples narrowing each partition search (1 on, 0 off)
    kTuneMergeBlockSort,   // CME_MERGE_BLOCK_SORT: keys-only 16384-key block sort, 1 LDS radix (4 digit passes), 0 merge network
    kTuneCount
};

// Current value of a knob (its environment variable or default until set).
long tune_get(TuneKey k);

}  // namespace cme
