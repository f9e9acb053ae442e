/*
 * pa.h -- C ABI of libpa.so, the MI355X (gfx950) pseudo-alignment engine.
 *
 * The reference (nyenyu12/BioInformatics-project-for-Shotgun-Metagenomics-
 * Pseudo-alignment-shotgun-, pure Python) has no FFI; its boundary for this
 * path is the Python API of src/kmer.py plus the dumpalign CLI.  Each entry
 * point below replaces one piece of that API (file:line in the reference):
 *
 *   pa_index_build           KmerReference.__init__ / _build_kmer_mapping   src/kmer.py:113-150
 *   pa_index_build_ex        the same, the align-side view deferred        src/kmer.py:113-133
 *   pa_index_reduce          KmerReference._filter_similar_genomes (pruning)  src/kmer.py:232-263
 *   pa_index_prepare         (the deferred view, before the first align)
 *   pa_index_prepare_ex      the same, sized for the reads the caller expects
 *   pa_params_effective      the filters a batch's align applies (Read.mean_quality /
 *                            kmer_quality thresholds no read can fail) src/kmer.py:394-408
 *   pa_index_lookup          KmerReference.get_kmer_references / __getitem__ src/kmer.py:284-298
 *   pa_index_class_genomes   (genome set of a k-mer, i.e. the keys of kmers[kmer]) src/kmer.py:130
 *   pa_index_positions       KmerReference.get_kmer_references (positions) and
 *                            get_kmer_and_reverse_references              src/kmer.py:292-298, 331-351
 *   pa_index_dumpref         KmerReference.get_summary ("Kmers" + Summary counts)
 *                            streamed as JSON text (dumpref)                src/kmer.py:300-329
 *   pa_index_extsim_stats    KmerReference._compute_genome_stats + the pairwise
 *                            intersections of _apply_greedy_filter          src/kmer.py:152-230
 *   pa_align                 PseudoAlignment.align_reads_from_container ->
 *                            Read.pseudo_align (counters only)              src/kmer.py:482-620
 *   pa_align_detail          the same, with per-read mapping type and
 *                            genomes_mapped_to (PseudoAlignment.reads)      src/kmer.py:542, 551-561
 *   pa_result_fetch          PseudoAlignment.get_summary inputs             src/kmer.py:622-657
 *   pa_align_batch           one-shot host-buffer form of pa_align
 *   pa_align_fastq_file      FASTAQFile + align_reads_from_container as one
 *                            device-parsed stream                          src/data_file.py:134-158,
 *                                                                          src/kmer.py:600-620
 *   pa_align_fastq_range     the same over a byte range of the file, one per device:
 *   pa_idsets_disjoint       the dumpalign job read-sharded over N GPUs     src/main.py:289-310
 *   pa_fastq_prefetch_start  the same with the file moved to the device in the
 *   pa_align_fastq_prefetched  background (overlaps the index build)       src/main.py:286-310
 *   pa_counters_reduce       the multi-GPU sum/min of PseudoAlignment counters
 *                            (read shards of one job); the
 *                            reference is single-process, so this has no
 *                            reference counterpart: it makes N per-rank
 *                            get_summary inputs equal to the one-process ones
 *                            src/kmer.py:622-657
 *   pa_parse_file/_text      FASTAFile / FASTAQFile -> FASTARecordContainer /
 *                            FASTAQRecordContainer.parse_records (host
 *                            threads, canonical subset of the grammar)     src/data_file.py:117-158,
 *                                                                          src/records.py:141-302
 *
 * Conventions
 *   - Every function returns PA_OK (0) or an error code; pa_last_error()
 *     gives a thread-local message.  The Python layer maps PA_EINVAL to
 *     ValueError and PA_ETYPE to TypeError, like src/kmer.py:501-510.
 *   - Buffers named seq/qual/genomes/read_off/... are HOST pointers; the
 *     library copies them.  Objects (pa_index, pa_reads, pa_result) own DEVICE
 *     memory on the device they were created on.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).  All work is
 *     stream-ordered; functions that return host data synchronize that stream.
 *   - Calls on one pa_index are not thread-safe with respect to each other.
 *   - Genome text must be uppercase ACGTN (the FASTA grammar,
 *     src/records.py:225-233); reads may contain any byte, but only ACGT
 *     windows can match (the FASTQ grammar restricts reads to ACGT,
 *     src/records.py:258-265).
 *   - Mapping types use the reference's enum values (src/kmer.py:41-47):
 *     1 UNMAPPED, 2 UNIQUELY_MAPPED, 3 AMBIGUOUSLY_MAPPED; 0 marks a read
 *     dropped by --min-read-quality (src/kmer.py:587-589: not in `reads`).
 */
#ifndef PA_H
#define PA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t pa_status;
#define PA_OK 0
#define PA_EINVAL 1        /* bad argument value (ValueError) */
#define PA_ETYPE 2         /* bad argument kind (TypeError) */
#define PA_ENOMEM 3        /* host or device allocation failed */
#define PA_EDEVICE 4       /* HIP runtime error */
#define PA_EUNSUPPORTED 5  /* e.g. k > PA_MAX_K */
#define PA_EINTERNAL 6     /* invariant violated (reported, never silent) */
#define PA_ENOTCANON 7     /* ingest: text outside the canonical FASTA/FASTQ subset (use the exact grammar) */
#define PA_EIO 8           /* ingest: file could not be opened / read */

#define PA_MAX_K 255       /* k-mers up to 255 bases: keys of up to 8 x 64-bit words */

#define PA_DROPPED 0
#define PA_UNMAPPED 1
#define PA_UNIQUELY_MAPPED 2
#define PA_AMBIGUOUSLY_MAPPED 3

/* pa_params.flags: which optional EXTQUALITY arguments are set (not None) */
#define PA_HAS_MIN_READ_QUALITY 1u
#define PA_HAS_MIN_KMER_QUALITY 2u
#define PA_HAS_MAX_GENOMES 4u

#define PA_NO_FIRST_KEY INT64_MAX  /* first_key of a genome never counted; all keys are < 2^63 */
/* first_key = (global read index << 20) | position in that read's
 * genomes_mapped_to list (<= G: a p-demoted list holds G* twice), so an index
 * holds at most PA_MAX_GENOMES genomes (pa_index_build: PA_EUNSUPPORTED above)
 * and read indices stay below 2^43. */
#define PA_MAX_GENOMES ((1u << 20) - 1)

typedef struct pa_index pa_index;
typedef struct pa_reads pa_reads;
typedef struct pa_result pa_result;

/* Arguments of Read.pseudo_align / align_reads_from_container (src/kmer.py:482-489, 600-606). */
typedef struct {
    int64_t m;                 /* unique threshold; < 0 -> PA_EINVAL (src/kmer.py:509-510) */
    int64_t p;                 /* ambiguity threshold; < 0 skips validation (src/kmer.py:469) */
    int64_t min_read_quality;  /* raw-ASCII mean, strict < (src/kmer.py:399, 587) */
    int64_t min_kmer_quality;  /* raw-ASCII window mean, strict < (src/kmer.py:408, 420) */
    int64_t max_genomes;       /* genomes per k-mer, strict > (src/kmer.py:425) */
    uint32_t flags;            /* PA_HAS_* */
    uint32_t reserved;
} pa_params;

/* "Statistics" of get_summary (src/kmer.py:627-637). */
typedef struct {
    uint64_t unique_mapped_reads;
    uint64_t ambiguous_mapped_reads;
    uint64_t unmapped_reads;
    uint64_t filtered_quality_reads;
    uint64_t filtered_quality_kmers;   /* windows, repeats included (quirk 4) */
    uint64_t filtered_hr_kmers;        /* windows, repeats included (quirk 4) */
} pa_stats;

typedef struct {
    uint32_t k;
    uint32_t n_genomes;
    uint32_t key_words;            /* 64-bit words per packed k-mer key */
    uint32_t slot_bytes;
    uint64_t n_kmers;              /* distinct k-mers (len(KmerReference.kmers)) */
    uint64_t n_multi_classes;      /* distinct genome sets with >= 2 genomes */
    uint64_t class_genome_entries;
    uint64_t table_slots;
    uint64_t table_bytes;
    uint64_t total_windows;        /* genome windows scanned by the build */
    uint64_t device_bytes;         /* all device memory held by the index */
} pa_index_info;

const char *pa_last_error(void);
const char *pa_version(void);
pa_status pa_device_count(int32_t *n);

/* ---- index (KmerReference) ---------------------------------------------- */

/* genomes: concatenated ASCII; genome_off: n_genomes+1 offsets (CSR). */
pa_status pa_index_build(int32_t device, const char *genomes, const uint64_t *genome_off, uint32_t n_genomes,
                         int64_t k, void *stream, pa_index **out);
/* The same with build flags.  PA_BUILD_DEFER_TILES: build the k-mer table and
 * the genome sets only; the align-side view (genome tiling, neighbour bits,
 * Bloom filter -- DESIGN.md section 3) is made by pa_index_prepare or by the
 * first pa_align / pa_align_detail call.  For an index that may only feed
 * pa_index_extsim_stats (KmerReference(..., filter_similar=True) builds, then
 * filters: src/kmer.py:113-133, 252-263) before it is rebuilt from the kept
 * genomes.  pa_index_build = pa_index_build_ex(..., 0, ...). */
#define PA_BUILD_DEFER_TILES 1u
/* PA_BUILD_COMPACT: the k-mer table at 2 slots per genome window (default 4;
 * for k <= 31: longer keys, and a table sized on the distinct k-mers, too
 * large for 2 per window, are not changed) -- builds faster, aligns
 * slightly slower (MI355X, round 6: C4 build 0.453 -> 0.395 s, its align pass
 * +4 %; C2 0.057 -> 0.048 s, +3 %).  For a job of fewer than
 * PA_COMPACT_READS_PER_BASE reads per genome base (the measured break-even,
 * 3-5): the CLI's dumpalign job, bench.py's job index.  Results never depend
 * on it.  Kept by pa_index_reduce when given again in its flags. */
#define PA_BUILD_COMPACT 2u
#define PA_COMPACT_READS_PER_BASE 3
pa_status pa_index_build_ex(int32_t device, const char *genomes, const uint64_t *genome_off, uint32_t n_genomes,
                            int64_t k, uint32_t flags, void *stream, pa_index **out);
/* Rebuild an index over some of its own genomes, in place: their 2-bit codes
 * are gathered on the device (nothing is concatenated or uploaded again), the
 * rest of the index is released and built anew -- the EXTSIM rebuild of
 * KmerReference(filter_similar=True), where the reference deletes the dropped
 * genomes from its dict (src/kmer.py:232-263).  keep: n_keep ascending genome
 * numbers (< n_genomes); flags as pa_index_build_ex.  On failure the index
 * holds nothing and may only be freed. */
pa_status pa_index_reduce(pa_index *idx, const uint32_t *keep, uint32_t n_keep, uint32_t flags, void *stream);
/* Make a deferred build's align-side view now, with the neighbour bits a
 * pa_index_prepare_ex or a FASTQ prefetch left pending (no-op otherwise);
 * returns when it is done. */
pa_status pa_index_prepare(pa_index *idx, void *stream);
/* The same for a job of about expected_reads reads (PA_READS_UNKNOWN: as
 * pa_index_prepare).  The one-substitution neighbour bits (DESIGN.md section
 * 3) cost time per genome base and save time per read: below the break-even
 * (PA_NB_READS_PER_KBASE[_2W/_3W] reads per 1000 genome bases) they are left out, and made by
 * the align that brings the reads aligned with this index past that point --
 * or by a later call of this function whose expected_reads (the reads still to
 * come) passes it.  Results never depend on them.  Returns when done. */
#define PA_READS_UNKNOWN UINT64_MAX
/* the measured break-even (bench.py neighbour_bits_breakeven, MI355X, round 6,
 * reverse-complement bits made lazily), reads per 1000 genome bases: keys of
 * one word (k <= 31; C2 1.45, C4 2.05, C5 2.80 reads per base), two words
 * (31 < k <= 63: c2k63 10.3) and three (63 < k <= 95: c2k75 18.5) */
#define PA_NB_READS_PER_KBASE 2500
#define PA_NB_READS_PER_KBASE_2W 10000
#define PA_NB_READS_PER_KBASE_3W 18000
pa_status pa_index_prepare_ex(pa_index *idx, uint64_t expected_reads, void *stream);
void pa_index_free(pa_index *idx);
pa_status pa_index_get_info(const pa_index *idx, pa_index_info *out);
/* n k-mers of length kmer_len packed back to back; cls_out[i] = class id or -1
 * if absent; size_out[i] = number of genomes containing it (0 if absent). */
pa_status pa_index_lookup(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len,
                          int64_t *cls_out, uint32_t *size_out, void *stream);
/* genome indices (ascending = FASTA order) of class `cls`; *n = class size. */
pa_status pa_index_class_genomes(const pa_index *idx, int64_t cls, uint32_t *genomes, uint32_t cap, uint32_t *n,
                                 void *stream);
/* Positions of n k-mers (kmer_len bases each, back to back) in the genomes:
 * every (query, genome, genome-local position) whose window holds the k-mer --
 * kmers[kmer] = {genome: positions} of the reference (src/kmer.py:140-150,
 * 292-298).  With PA_POS_REVERSE also every window holding its reverse
 * complement, unless that is the k-mer itself (get_kmer_and_reverse_references,
 * src/kmer.py:331-351); such hits carry PA_POS_RC_BIT in `query`.  A k-mer of
 * another length than the index's k, or with anything but A/C/G/T, has none.
 * Hits are sorted by (query, strand, genome, position); *n_hits = all of them,
 * of which the first min(cap, *n_hits) are written (hits may be NULL to count).
 * Genomes are numbered as built (after EXTSIM: the kept genomes). */
#define PA_POS_REVERSE 1u
#define PA_POS_RC_BIT 0x80000000u
typedef struct {
    uint32_t query;     /* query index | PA_POS_RC_BIT for a reverse-complement hit */
    uint32_t genome;
    uint64_t position;  /* window start within the genome */
} pa_kmer_hit;
pa_status pa_index_positions(const pa_index *idx, const char *kmers, uint64_t n, uint32_t kmer_len, uint32_t flags,
                             pa_kmer_hit *hits, uint64_t cap, uint64_t *n_hits, void *stream);
/* EXTSIM inputs at identifier-group granularity (group_of[n_genomes]):
 * total[a] = distinct k-mers touching group a, uniq[a] = k-mers contained in
 * exactly one genome which belongs to a, inter[a*n_groups+b] = k-mers touching
 * both groups a != b. */
pa_status pa_index_extsim_stats(const pa_index *idx, const uint32_t *group_of, uint32_t n_groups, uint64_t *total,
                                uint64_t *uniq, uint64_t *inter, void *stream);

/* ---- reads ------------------------------------------------------------------ */

pa_status pa_reads_upload(int32_t device, const uint8_t *seq, const uint8_t *qual, const uint64_t *read_off,
                          uint64_t n_reads, void *stream, pa_reads **out);
/* Synthetic fixed-length forward-strand reads sampled on the device from the
 * index's genomes (read i = global read first_read + i; deterministic in seed). */
pa_status pa_reads_synthesize(const pa_index *idx, uint64_t n_reads, uint32_t read_len, uint64_t first_read,
                              uint64_t seed, double sub_rate, void *stream, pa_reads **out);
/* The same with a share of reverse-complemented reads (rc_rate: the reference
 * looks up forward k-mers only, so these mostly go unmapped) and of reads of
 * uniform random bases (foreign_rate: an organism absent from the index); the
 * rest forward.  rc_rate + foreign_rate <= 1.  (The robustness workload.) */
pa_status pa_reads_synthesize_mix(const pa_index *idx, uint64_t n_reads, uint32_t read_len, uint64_t first_read,
                                  uint64_t seed, double sub_rate, double rc_rate, double foreign_rate, void *stream,
                                  pa_reads **out);
pa_status pa_reads_info(const pa_reads *reads, uint64_t *n_reads, uint64_t *n_bases, uint32_t *max_len);
/* The filter arguments a pa_align of this batch applies (out, may alias in):
 * a --min-read-quality / --min-kmer-quality at or below the batch's smallest
 * quality byte can filter nothing (strict <, src/kmer.py:420, 587; quirk 5)
 * and is dropped from the pass -- its flag cleared, the counters unchanged.
 * q_min (nullable): that byte (255: no quality bytes). */
pa_status pa_params_effective(const pa_reads *reads, const pa_params *in, pa_params *out, int32_t *q_min,
                              void *stream);
/* copy reads [first, first+count) back to the host (seq/qual: n_bases of that range) */
pa_status pa_reads_download(const pa_reads *reads, uint64_t first, uint64_t count, uint8_t *seq, uint8_t *qual,
                            uint64_t *read_off, void *stream);
void pa_reads_free(pa_reads *reads);

/* ---- results (PseudoAlignment counters) ------------------------------------- */

pa_status pa_result_create(const pa_index *idx, pa_result **out);
pa_status pa_result_reset(pa_result *res, void *stream);
/* any output pointer may be NULL; per-genome arrays hold n_genomes entries */
pa_status pa_result_fetch(const pa_result *res, pa_stats *stats, uint64_t *unique_reads, uint64_t *ambiguous_reads,
                          uint64_t *first_key, void *stream);
/* Device views for collectives: sum block = [6 stats][G unique][G ambiguous]
 * (reduce with SUM), min block = [G first_key] (reduce with MIN). */
pa_status pa_result_device_view(pa_result *res, uint64_t **sum_block, uint64_t *n_sum, uint64_t **min_block,
                                uint64_t *n_min);
/* Stream-ordered device-to-device copies of the two blocks to / from caller
 * device buffers (e.g. torch tensors reduced with RCCL); either pointer may be
 * NULL.  Values fit int64: counts < 2^63, first keys < 2^63 (PA_NO_FIRST_KEY). */
pa_status pa_result_copy_out(const pa_result *res, void *sum_dst, void *min_dst, void *stream);
pa_status pa_result_copy_in(pa_result *res, const void *sum_src, const void *min_src, void *stream);
/* Overwrite the two blocks from HOST arrays ([6 + 2G] sums, [G] first keys, as
 * pa_result_fetch's order: stats, unique, ambiguous); returns when copied.
 * The host-side reduction of read shards (dumpalign over N GPUs). */
pa_status pa_result_load(pa_result *res, const uint64_t *sum_block, const uint64_t *min_block);
void pa_result_free(pa_result *res);

/* ---- alignment ---------------------------------------------------------------- */

/* Accumulates into `acc`.  read_index_base = global index of reads[0] (orders
 * the Summary keys by first appearance, quirk 9). */
pa_status pa_align(const pa_index *idx, const pa_reads *reads, const pa_params *params, uint64_t read_index_base,
                   pa_result *acc, void *stream);
/* Per-read results.  read_type[n], filtered_kmers[n], redundant_kmers[n],
 * list_off[n+1] (host).  lists may be NULL to query *list_total first. */
pa_status pa_align_detail(const pa_index *idx, const pa_reads *reads, const pa_params *params, uint8_t *read_type,
                          uint32_t *filtered_kmers, uint32_t *redundant_kmers, uint64_t *list_off, uint32_t *lists,
                          uint64_t list_cap, uint64_t *list_total, void *stream);
/* upload + pa_align + fetch for host buffers (stats and per-genome arrays accumulate: +=, min) */
pa_status pa_align_batch(const pa_index *idx, const uint8_t *seq, const uint8_t *qual, const uint64_t *read_off,
                         uint64_t n_reads, uint64_t read_index_base, const pa_params *params, pa_stats *stats,
                         uint64_t *unique_reads, uint64_t *ambiguous_reads, uint64_t *first_key, void *stream);

/* A FASTQ file straight into the align pass (FASTAQFile(path).container +
 * PseudoAlignment.align_reads_from_container, src/data_file.py:134-158,
 * src/records.py:245-302, src/kmer.py:600-620): the host reads the file in
 * windows of window_bytes (0: 128 MiB; threads readers, or zlib for ".gz") into
 * pinned buffers; the DEVICE finds the records, checks them against the
 * grammar, hashes the ids into a duplicate set, packs the read columns and
 * aligns each window while the host reads the next.  Record i of the file is
 * global read read_index_base + i; *n_reads = records.  PA_ENOTCANON: the
 * file is outside the device-parsed subset of the grammar (LF line ends, "+"
 * lines, ids without outer blanks, see csrc/pa_fastq.hip), holds a duplicate
 * id or no record -- `acc` then holds a partial sum: reset it and parse the
 * file the exact way (which also raises the reference's errors). */
pa_status pa_align_fastq_file(const pa_index *idx, const char *path, const pa_params *params,
                              uint64_t read_index_base, pa_result *acc, int32_t threads, uint64_t window_bytes,
                              void *stream, uint64_t *n_reads);

/* pa_align_fastq_file over the byte range [offset, offset + length) of a plain
 * (not gzip) FASTQ file, read as if it were the whole file: the shard of one
 * device in a read-sharded job (the dumpalign CLI with PA_GPUS = N).  The
 * range must start at a record's '@' and end after a record's last line feed
 * (or at the end of the file).  read_index_base orders the shards' records:
 * any base at least as large as the previous shard's base + its record count
 * keeps the Summary key order of one pass over the file (e.g. the range's
 * byte offset: every record takes more than one byte).  ids (nullable): the
 * range's read-id hashes, for pa_idsets_disjoint -- the duplicate-id check
 * (DuplicateRecordError, src/records.py:290-302) across ranges; a duplicate
 * within the range is PA_ENOTCANON as in pa_align_fastq_file. */
typedef struct pa_idset pa_idset;
pa_status pa_align_fastq_range(const pa_index *idx, const char *path, uint64_t offset, uint64_t length,
                               const pa_params *params, uint64_t read_index_base, pa_result *acc, int32_t threads,
                               uint64_t window_bytes, void *stream, uint64_t *n_reads, pa_idset **ids);
/* *disjoint = 1 when no read-id hash is in two of the sets (else 0: a duplicate
 * id across shards, or a 2^-64 hash collision -- parse the file the exact way,
 * which decides and raises the reference's error).  Checked on `device`. */
pa_status pa_idsets_disjoint(const pa_idset *const *sets, uint32_t n_sets, int32_t device, int32_t *disjoint);
void pa_idset_free(pa_idset *ids);

/* The same as one device-resident step: pa_fastq_prefetch_start begins moving
 * the (plain, not gzip) FASTQ file into device memory on a background thread
 * (parallel positional reads into a pinned ring, copies in file order) and
 * returns at once, so that the copy overlaps the caller's FASTA parse and
 * index build (the dumpalign CLI starts it first); pa_align_fastq_prefetched
 * then parses and aligns the file window by window (window_bytes, 0: 128 MiB)
 * as the bytes land, with the records, errors and PA_ENOTCANON of
 * pa_align_fastq_file.  PA_EUNSUPPORTED for ".gz" paths (use
 * pa_align_fastq_file).  One align per prefetch; free it afterwards. */
typedef struct pa_fastq_prefetch pa_fastq_prefetch;
pa_status pa_fastq_prefetch_start(const char *path, int32_t device, int32_t threads, uint64_t window_bytes,
                                  pa_fastq_prefetch **out);
pa_status pa_align_fastq_prefetched(const pa_index *idx, pa_fastq_prefetch *prefetch, const pa_params *params,
                                    uint64_t read_index_base, pa_result *acc, void *stream, uint64_t *n_reads);
void pa_fastq_prefetch_free(pa_fastq_prefetch *prefetch);

/* dumpref (KmerReference.get_summary, src/kmer.py:300-329; CLI src/main.py:121-158):
 * the "Kmers" object of the summary written to file descriptor fd as
 * json.dumps(indent=4) text at nesting level 1 ("{" ... "\n    }", or "{}"),
 * from the device index: k-mers in the reference's insertion order (first
 * occurrence in FASTA order), each with its genomes' descriptions and sorted
 * positions.  desc_of[g] numbers genome g's description (desc_json[d]: its
 * JSON string literal, quotes included); genomes sharing a description merge
 * as dict keys do.  keep[g] (NULL: all): genomes left by EXTSIM -- the index
 * must then hold ALL genomes, so that the surviving k-mers keep the full
 * build's order (src/kmer.py:232-245).  Per description: k-mers held by it
 * with one genome / several (unique_kmers / multi_mapping_kmers), its rank of
 * first appearance (the Summary key order; UINT64_MAX if absent) and the last
 * genome met with it (its total_bases); *n_kmers = k-mers written. */
pa_status pa_index_dumpref(const pa_index *idx, const uint8_t *keep, const uint32_t *desc_of, uint32_t n_desc,
                           const char *const *desc_json, int32_t fd, int32_t threads, uint64_t *desc_unique,
                           uint64_t *desc_multi, uint64_t *desc_order, uint32_t *desc_last_genome, uint64_t *n_kmers);

/* Start the HIP runtime and device `device` on a background thread and return
 * at once (a command-line run calls it first, so the runtime's start-up of
 * ~0.15 s overlaps its imports and FASTA parse); later calls wait for it as
 * for any runtime start.  Always PA_OK (errors surface at the first real call). */
pa_status pa_runtime_start(int32_t device);

/* ---- multi-GPU reduce (RCCL over xGMI) ------------------------------------------- */

/* One process per GPU, each aligning its own read shard with GLOBAL read
 * indices (read_index_base), then ONE in-place all-reduce of every rank's
 * pa_result: the sum block with ncclSum, the first-key block with ncclMin
 * (uint64).  Afterwards every rank's pa_result holds the job's counters, and
 * pa_result_fetch gives exactly what one process aligning all reads would
 * (Summary key order included).  RCCL is opened at the first call
 * (PA_RCCL_LIBRARY or librccl.so.1); PA_EUNSUPPORTED if it cannot be.
 * `comm` is an ncclComm_t -- from pa_comm_init, or any RCCL communicator of
 * the job's ranks (e.g. the one a framework already made).  Stream-ordered on
 * `stream`; collective: every rank must call it. */
#define PA_COMM_ID_BYTES 128
pa_status pa_comm_unique_id(uint8_t *id /* [PA_COMM_ID_BYTES], rank 0; share it with the others */);
pa_status pa_comm_init(int32_t device, int32_t nranks, int32_t rank, const uint8_t *id, void **comm);
pa_status pa_comm_free(void *comm);
/* ranks in the communicator (ncclCommCount): what a job's reduce really spans */
pa_status pa_comm_count(void *comm, int32_t *nranks);
pa_status pa_counters_reduce(pa_result *res, void *comm, void *stream);

/* ---- profiling ------------------------------------------------------------------ */

/* When enabled, pa_align records HIP events around its main kernel on the
 * stream it launches on; pa_profile_read synchronizes and returns the summed
 * main-kernel milliseconds, launch count, and the reads that took the exact
 * (deferred) path since the last read. */
pa_status pa_profile_enable(pa_index *idx, int32_t enable);
pa_status pa_profile_read(pa_index *idx, double *main_ms, uint64_t *launches, uint64_t *deferred_reads);
/* The same events per kernel of the align pass (each launch bracketed by its
 * own pair on the launch stream): ms[PA_PROF_KERNELS] summed milliseconds and
 * launches[PA_PROF_KERNELS] launch counts since the last call, indexed by
 * PA_PROF_*.  Independent of pa_profile_read (either may be read first). */
#define PA_PROF_QUALITY 0   /* k_quality_masks */
#define PA_PROF_LANE 1      /* k_align_lane (the dominant kernel) */
#define PA_PROF_LANE_NA 2   /* k_align_lane_na */
#define PA_PROF_WAVE 3      /* k_align_fast */
#define PA_PROF_EXACT 4     /* k_align_exact */
#define PA_PROF_LANE_RC 5   /* k_align_lane_rc */
#define PA_PROF_RC_SEEDS 6  /* k_rc_seeds */
#define PA_PROF_KERNELS 7
pa_status pa_profile_read_kernels(pa_index *idx, double *ms, uint64_t *launches);

/* ---- device memory -------------------------------------------------------------- */

/* Buffers of 256 MiB and more (tables, tiles, read columns) come from slabs
 * the library keeps per device and reuses after a free (csrc/pa_mem.cpp: the
 * driver reclaims given-back memory at ~60 GB/s, which stalled rebuilds such as
 * EXTSIM's index of the kept genomes).  pa_mem_trim gives the idle slabs of
 * `device` (-1: every device) back to the driver, for a process that needs the
 * memory elsewhere; *released (may be NULL) = bytes given back.  Allocations
 * that cannot be met otherwise trim by themselves.  No reference counterpart
 * (the reference holds its index in Python dicts). */
pa_status pa_mem_trim(int32_t device, uint64_t *released);

/* ---- ingest (host only, no device) ---------------------------------------------- */

/* Multi-threaded parse of FASTA (kind PA_FASTA) or FASTQ (PA_FASTQ) text into
 * column buffers, for the canonical subset of the reference grammar
 * (src/records.py:141-302; csrc/pa_ingest.cpp states the subset).  Returns
 * PA_ENOTCANON for any text outside it -- including every text the reference
 * rejects (no records, unparsed data, duplicate ids, length mismatch) -- so
 * that the caller parses it with the exact grammar, which reproduces the
 * reference's acceptance and errors.  pa_parse_file reads plain files by mmap
 * and ".gz" files as pa_gz_inflate_file does; PA_EIO if the file cannot be read.
 * A pa_seqset holds n records: FASTA genomes with whitespace removed and
 * stripped descriptions; FASTQ sequences, qualities and stripped ids. */
#define PA_FASTA 0
#define PA_FASTQ 1
typedef struct pa_seqset pa_seqset;
/* universal_newlines: 1 = the text was read from a file in text mode by the
 * reference (CRLF / lone final CR are line breaks), 0 = raw text (parse_records(str)) */
pa_status pa_parse_text(int32_t kind, const char *text, uint64_t len, int32_t threads, int32_t universal_newlines,
                        pa_seqset **out);
pa_status pa_parse_file(int32_t kind, const char *path, int32_t threads, pa_seqset **out);
/* n_bases: total sequence bytes; name_bytes: names joined by '\n' (one after each name) */
pa_status pa_seqset_sizes(const pa_seqset *set, uint64_t *n_records, uint64_t *n_bases, uint64_t *name_bytes);
/* seq[n_bases], qual[n_bases] (FASTQ; may be NULL), off[n_records + 1] (CSR), names[name_bytes] (may be NULL) */
pa_status pa_seqset_export(const pa_seqset *set, uint8_t *seq, uint8_t *qual, uint64_t *off, char *names);
void pa_seqset_free(pa_seqset *set);

/* The text of a ".gz" file, as gzip.open(path).read() returns it
 * (src/data_file.py:123-125), inflated on `threads` host threads: BGZF members
 * in parallel, any other gzip member by chunks whose block boundaries are
 * found by search (csrc/pa_pgz.cpp); every member's CRC-32 and size checked.
 * *n = the text's length; PA_EINVAL if it exceeds cap, PA_ENOTCANON for data
 * gzip.open would not read cleanly (the caller then raises the reference's
 * error through Python's gzip), PA_EIO if the file cannot be opened. */
pa_status pa_gz_inflate_file(const char *path, int32_t threads, uint8_t *dst, uint64_t cap, uint64_t *n);

#ifdef __cplusplus
}
#endif

#endif /* PA_H */
