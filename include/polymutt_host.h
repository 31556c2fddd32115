/*
 * polymutt_host.h -- C ABI of the host-side helpers that sit beside the engine in libpolymutt.so:
 * pedigree loading (Merlin .dat/.ped with polyMutt's ordering), GLF section/site reading into the
 * dense blocks pm_engine_run consumes, and the synthetic workload generator.
 *
 * These replace, for FFI callers, the reference's Pedigree::Prepare/Load (core/PedigreeLoader.cpp),
 * PedigreeGLF::SetPedGLF/Move2NextSection/Move2NextBaseEntry (src/PedigreeGLF.cpp:117-324) and
 * glfHandler (core/glfHandler.cpp).  Errors: NULL / negative return, message in pm_last_error().
 */
#ifndef POLYMUTT_HOST_H
#define POLYMUTT_HOST_H
#include "polymutt_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pmh_pedigree pmh_pedigree;
pmh_pedigree *pmh_pedigree_load(const char *dat_file, const char *ped_file);
/* Fills *out with pointers owned by the handle (valid until pmh_pedigree_free). */
int pmh_pedigree_view(const pmh_pedigree *p, pm_pedigree *out);
const char *pmh_pedigree_pid(const pmh_pedigree *p, int32_t person);
const char *pmh_pedigree_famid(const pmh_pedigree *p, int32_t family);
int32_t pmh_pedigree_is_nuclear(const pmh_pedigree *p, int32_t family);
void pmh_pedigree_free(pmh_pedigree *p);

/* GLF reading: one GLF per person through the index file ("key path" lines; key = GLF_Index). */
typedef struct pmh_glf_reader pmh_glf_reader;
pmh_glf_reader *pmh_glf_open(const pmh_pedigree *p, const char *glf_index_file);
/* Advance to the next section; returns 1 and copies the label (NUL-terminated) or 0 at end. */
int pmh_glf_next_section(pmh_glf_reader *r, char *label, int32_t label_cap, int32_t *max_position);
/* Read up to max_sites sites of the current section into dense rows; returns the count (0 = end). */
int pmh_glf_read_sites(pmh_glf_reader *r, int32_t max_sites, int32_t *pos, uint8_t *ref, uint8_t *pl, uint32_t *dm);
void pmh_glf_close(pmh_glf_reader *r);

/* The polymutt command line (src/main.cpp:57-627) on the HIP engine; returns the exit code.
 * world > 1: this process is shard `rank` of a multi-GPU run (one process per GPU, launched by
 * polymutt_amd/launch.py): it analyses a contiguous position range of every section and calls
 * allgather(ctx, send, n, recv) -- recv receives world x n int64, rank-major -- once per section and
 * once at the end; rank 0 prints the summed summaries and writes the merged VCF.  world == 1 with a non-null
 * allgather runs the same sharded protocol over one rank (the exchange on the device's collective, e.g. RCCL at
 * world 1); world == 1 with a null allgather is the plain one-process CLI.  device >= 0 overrides --gpu.  allgather
 * returns 0 on success. */
typedef int (*pmh_allgather_fn)(void *ctx, const int64_t *send, int32_t n, int64_t *recv);
int pmh_run_polymutt(int argc, char **argv, int32_t rank, int32_t world, int32_t device, pmh_allgather_fn allgather,
                     void *ctx);

/* Synthetic workload.  shape: "quad", "trio", "ext10" (3-generation, 10 members),
 * "roof" (double-roof 8 members), "roof2" (12 members: a type-3 peel with a marriage partial), "mixed"
 * (alternating trio/quad), "single" (unrelated singletons), "quadext" (quads with an ext10 at families
 * 256, 513, ...); "<shape>+dn" plants de novo calls. */
int pmh_synth_write_dataset(const char *dir, const char *shape, int32_t n_fam, int32_t n_sites, uint64_t seed);
/* Host generation of the same dense block pm_engine_synth produces on the device. */
int pmh_synth_block(const pm_pedigree *ped, int32_t n, uint64_t seed, uint64_t site_offset, uint8_t *pl, uint32_t *dm, uint8_t *ref);

#ifdef __cplusplus
}
#endif
#endif
