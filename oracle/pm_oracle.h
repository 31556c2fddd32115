/*
 * oracle/pm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-site family-likelihood model (genome-vendor/polymutt v0.13),
 * used solely as the parity checker for the HIP engine (tests/, __graft_entry__.smoke(), and
 * bench.py's cpu_baseline leg).  The product never links this code.
 *
 * Pinning: the restatement is checked against (1) the reference's committed goldens
 * (example/test.out.vcf, test.denovo.out.vcf, test.out.vcfa) and (2) per-site intermediates dumped by
 * oracle/_ref/pm_ref, a driver of ours linked against the reference's own objects (oracle/ref/).
 * It follows the reference's serial operation order (family loop, sums, products) and uses glibc
 * log10/exp10/pow exactly where the reference does, so it is bit-identical to the reference.
 */
#ifndef PM_ORACLE_H
#define PM_ORACLE_H
#include "../include/polymutt_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pmo_ctx pmo_ctx;

pmo_ctx *pmo_create(const pm_pedigree *ped, const pm_params *par);
void pmo_destroy(pmo_ctx *c);
void pmo_begin_section(pmo_ctx *c, int32_t chrom);
/* famlk[0]'s stale posterior state (see pm_engine_set_posterior_carry). */
void pmo_set_posterior_carry(pmo_ctx *c, int32_t seen);
double pmo_poly_prior(const pmo_ctx *c);

/* One site of main.cpp:327-594.  calls[n_person] is written when res->emit != 0.
 * Returns 0, or PM_EBRENT if Brent hit ITMAX (reference: numerror exit). */
int pmo_site(pmo_ctx *c, const uint8_t *pl, const uint32_t *dm, int32_t ref, pm_site_result *res, pm_geno_call *calls);

/* Building blocks exposed for unit tests. */
double pmo_objective(pmo_ctx *c, const uint8_t *pl, int32_t a1, int32_t a2, double freq, int32_t denovo);
double pmo_poly_loglik(pmo_ctx *c, const uint8_t *pl, int32_t a1, int32_t a2, int32_t denovo, double *min_out, int32_t *evals);
void pmo_counters(const pmo_ctx *c, pm_counters *out);
const double *pmo_geno_mut_matrix(const pmo_ctx *c);   /* 10x10 row-major */

#ifdef __cplusplus
}
#endif
#endif
