/*
 * oracle/pm_oracle.c -- TEST INFRASTRUCTURE ONLY (see pm_oracle.h).
 *
 * Serial CPU restatement of the reference per-site model.  Every function cites the reference
 * file:line it restates (paths relative to the reference root).  Build: plain C99, no -march, no FMA
 * contraction (the reference is generic x86-64 SSE2 code, src/Makefile:1), glibc libm.
 */
#define _GNU_SOURCE
#include "pm_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MALE 1
#define FEMALE 2
#define ITMAX 200              /* core/MathConstant.h:16 */
#define ZEPS 3.0e-10           /* core/MathConstant.h:18 */
#define CGOLD 0.38196601       /* core/MathConstant.h:23 */

/* Mutable state the reference keeps in its seven FamilyLikelihoodSeq objects across sites
 * (main.cpp:248).  Only what changes observable output is kept. */
typedef struct {
  int a1, a2, g11, g12, g22;   /* SetAlleles, NucFamGenotypeLikelihood.cpp:89-97 */
  int sex;                     /* member `sex` read by likelihoodONEKid (:1202-1264) -- stale by design */
  int is_mono;                 /* member isMono read by CalcParentMarginal (:1064) */
  double min, fmin;            /* ScalarMinimizer::min/fmin, persists between sites */
  long evals;
} lkobj;

#define PMO_MAXT 64
struct pmo_scratch {
  double parentGLF[9], parentPrior[9], parentMarginal[9];
  double *partials;            /* [max fam size][10] */
  double mp[64][10][10];       /* marriage partials, keyed below */
  int mpkey[64][2], nmp;
};

struct pmo_ctx {
  pm_pedigree ped;
  int32_t *fam_start, *fam_founders, *fam_kind, *peel_start;
  int8_t *sex, *is_founder;
  pm_peel_step *steps;
  pm_params par;
  int chrom, isX, isY, isMT;
  int itmax;   /* ITMAX (200); PM_TEST_ITMAX lowers it, as for the engine (failure-path tests) */
  double prior;                /* GetPolyPrior() of the section */
  double lktab[256];           /* core/BaseQualityHelper.cpp:13 */
  double M[10][10];            /* GenotypeMutationModel::genoMutMatrix */
  double T10[10][10][10];      /* FamilyLikelihoodES::transmission */
  double T10dn[10][10][10];    /* FamilyLikelihoodES::transmission_denovo */
  double TBA[5][3][3][3];      /* transmission_BA, _CHRX_2Female, _CHRX_2Male, _CHRY, _MITO */
  lkobj lk[7];
  int denovo;                  /* par->denovo as currently seen by the objective (main.cpp:569-572 toggles it) */
  int unrelated;               /* --quick_call MakeUnrelated() in effect (FamilyLikelihoodSeq.cpp:54-59) */
  int any_postprob;            /* famlk[0].CalcPostProb has run at least once (sets the stale sex) */
  int vcf_objective;           /* Brent objective is FamilyLikelihoodSeq_VCF::f (vcf_mode) */
  const uint8_t *pl;           /* current site */
  const uint32_t *dm;
  int refBase;
  pm_counters cnt;
  /* scratch of the objective, one per OpenMP thread (pmo_site runs the reference's `omp parallel sections` over the
   * allele configurations when built with -fopenmp, main.cpp:361-393, 401-426, 439-495, 501-535) */
  struct pmo_scratch *scr;
  double *postv;               /* [n_person][10] */
  int *best;
  int8_t *label;
  double *dosage;
};

static int GI(int b1, int b2) { /* glfHandler::GenotypeIndex, core/glfHandler.h:102-106 */
  return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2);
}
static int poly_ts(int r) { static const int t[5] = {0, 3, 4, 1, 2}; return (r >= 1 && r <= 4) ? t[r] : 0; }   /* src/PedigreeGLF.h:14-29 */
static int poly_tv1(int r) { static const int t[5] = {0, 2, 1, 2, 1}; return (r >= 1 && r <= 4) ? t[r] : 0; }  /* :30-42 */
static int poly_tv2(int r) { static const int t[5] = {0, 4, 3, 4, 3}; return (r >= 1 && r <= 4) ? t[r] : 0; }  /* :43-53 */
static double sign_(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }   /* core/MathConstant.h:31 */

static inline int fam_count(const pmo_ctx *c, int f) { return c->fam_start[f + 1] - c->fam_start[f]; }
static inline int fam_founders(const pmo_ctx *c, int f) { return c->unrelated ? fam_count(c, f) : c->fam_founders[f]; }
/* Family::isNuclear (core/PedigreeFamily.h:29-30) with MakeUnrelated applied */
static inline int fam_nuclear(const pmo_ctx *c, int f) { return !c->unrelated && c->fam_kind[f] == PM_FAM_NUCLEAR; }
static inline int fam_allfounders(const pmo_ctx *c, int f) { return fam_count(c, f) == fam_founders(c, f); }
static inline double pen(const pmo_ctx *c, int person, int g) { return c->lktab[c->pl[person * 10 + g]]; }
static inline struct pmo_scratch *SC(const pmo_ctx *c) {   /* this thread's scratch (unique across nested teams) */
#ifdef _OPENMP
  int t = 0;
  for (int l = 1, lv = omp_get_level(); l <= lv; l++) t = t * omp_get_team_size(l) + omp_get_ancestor_thread_num(l);
  return &c->scr[t < PMO_MAXT ? t : 0];
#else
  return &c->scr[0];
#endif
}

static void set_alleles(const pmo_ctx *c, lkobj *o, int a1, int a2) {
  (void)c; o->a1 = a1; o->a2 = a2; o->g11 = GI(a1, a1); o->g12 = GI(a1, a2); o->g22 = GI(a2, a2);
}

/* ---------------- mutation model / transmission tables ---------------- */
static void build_tables(pmo_ctx *c) {
  for (int i = 0; i <= 255; i++) c->lktab[i] = pow(0.1, i * 0.1);   /* core/BaseQualityHelper.cpp:12-13 */
  if (c->par.vcf_mode)   /* FamilyLikelihoodSeq_VCF::PL2LK_table, src/FamilyLikelihoodSeq_VCF.cpp:21-22 (PL > 255 clamps, :57-63) */
    for (int i = 0; i <= 255; i++) c->lktab[i] = pow(10, -(double)i / 10.0);
  /* AlleleMutationModel::SetAlleleMutMatrix, src/MutationModel.cpp:15-30 */
  double mu = c->par.denovo_mut_rate, tstv = c->par.denovo_tstv, A[4][4];
  for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) A[i][j] = (i == j) ? 1 - mu : (1 - mu) / 3;
  if (tstv != 0.0) {
    A[0][2] = A[2][0] = A[1][3] = A[3][1] = mu / 3 * (3 - 3 / (1 + tstv));
    A[0][1] = A[0][3] = A[1][0] = A[1][2] = A[2][1] = A[2][3] = A[3][0] = A[3][2] = mu / 3 * (0.5 / (1 + tstv) * 3);
  }
  /* GenotypeMutationModel::SetGenoMutMatrix, src/MutationModel.cpp:49-90 */
  double R[16][16];
  int from = -1;
  for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) {
    from++; int to = -1;
    for (int ii = 0; ii < 4; ii++) for (int jj = 0; jj < 4; jj++) { to++; R[from][to] = A[i][ii] * A[j][jj]; }
  }
  static const int h1[6] = {2, 3, 4, 7, 8, 12}, h2[6] = {5, 9, 13, 10, 14, 15};
  for (int i = 0; i < 6; i++) for (int j = 0; j < 16; j++) R[j][h1[i] - 1] += R[j][h2[i] - 1];
  static const int un[10] = {1, 2, 3, 4, 6, 7, 8, 11, 12, 16};
  for (int i = 0; i < 10; i++) for (int j = 0; j < 10; j++) c->M[i][j] = R[un[i] - 1][un[j] - 1];
  /* FamilyLikelihoodES::SetTransmissionMatrix, src/FamilyLikelihoodES.cpp:752-785 */
  memset(c->T10, 0, sizeof(c->T10));
  for (int i = 1; i <= 4; i++) for (int j = i; j <= 4; j++) {
    int x = GI(i, j);
    for (int k = 1; k <= 4; k++) for (int m = k; m <= 4; m++) {
      int y = GI(k, m), g[4] = {GI(i, k), GI(i, m), GI(j, k), GI(j, m)};
      for (int t = 0; t < 4; t++) c->T10[x][y][g[t]] += 0.25;
    }
  }
  /* SetTransmissionMatrix_denovo, :787-810 */
  for (int i = 0; i < 10; i++) for (int j = 0; j < 10; j++) for (int k = 0; k < 10; k++) {
    double s = .0;
    for (int m = 0; m < 10; m++) s += c->T10[i][j][m] * c->M[m][k];
    c->T10dn[i][j][k] = s;
  }
  /* SetTransmissionMatrix_BA* tables, :812-924 (index: 0 auto, 1 X->female, 2 X->male, 3 Y, 4 MT) */
  static const double ba[5][27] = {
    {1,0,0, .5,.5,0, 0,1,0,  .5,.5,0, .25,.5,.25, 0,.5,.5,  0,1,0, 0,.5,.5, 0,0,1},
    {1,0,0, .5,.5,0, 0,1,0,  0,0,0, 0,0,0, 0,0,0,          0,1,0, 0,.5,.5, 0,0,1},
    {1,0,0, .5,0,.5, 0,0,1,  0,0,0, 0,0,0, 0,0,0,          1,0,0, .5,0,.5, 0,0,1},
    {1,0,0, 1,0,0, 1,0,0,    0,0,0, 0,0,0, 0,0,0,          0,0,1, 0,0,1, 0,0,1},
    {1,0,0, 0,0,0, 0,0,1,    0,0,0, 0,0,0, 0,0,0,          1,0,0, 0,0,0, 0,0,1}};
  for (int t = 0; t < 5; t++) for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) for (int k = 0; k < 3; k++)
    c->TBA[t][i][j][k] = ba[t][i * 9 + j * 3 + k];
}

/* ---------------- priors ---------------- */
/* SetPolyPrior / _chrX / _chrY / _MT, NucFamGenotypeLikelihood.cpp:231-304 */
static double poly_prior(const pmo_ctx *c) {
  int n;
  if (c->isX) n = c->ped.female_founders * 2 + c->ped.male_founders;
  else if (c->isY) n = c->ped.male_founders;
  else if (c->isMT) n = c->ped.n_founders;
  else n = 2 * c->ped.n_founders;
  double p = 0;
  for (int i = 1; i <= n; i++) p += 1.0 / i;
  return p * c->par.theta;
}

/* SetParentPrior, NucFamGenotypeLikelihood.cpp:318-368 (pow(freq,k) is __builtin_powi under gnu++98) */
static void set_parent_prior(pmo_ctx *c, const lkobj *o, double f) {
  double *p = SC(c)->parentPrior;
  if (c->ped.n_fam > 1 || o->is_mono) {
    if (!c->isX && !c->isY && !c->isMT) {
      p[0] = (f * f) * (f * f);
      p[1] = f * f * f * (1 - f) * 2;
      p[2] = f * f * (1 - f) * (1 - f);
      p[3] = f * (1 - f) * 2 * f * f;
      p[4] = f * (1 - f) * 2 * f * (1 - f) * 2;
      p[5] = f * (1 - f) * 2 * (1 - f) * (1 - f);
      p[6] = (1 - f) * (1 - f) * f * f;
      p[7] = (1 - f) * (1 - f) * f * (1 - f) * 2;
      p[8] = (1 - f) * (1 - f) * (1 - f) * (1 - f);
    }
    if (c->isX) {
      p[0] = (f * f) * f; p[1] = f * f * (1 - f) * 2; p[2] = f * (1 - f) * (1 - f);
      p[3] = 0; p[4] = 0; p[5] = 0;
      p[6] = (1 - f) * f * f; p[7] = (1 - f) * f * (1 - f) * 2; p[8] = (1 - f) * (1 - f) * (1 - f);
    }
    if (c->isY) {
      p[0] = f; p[1] = f; p[2] = f; p[3] = 0; p[4] = 0; p[5] = 0; p[6] = (1 - f); p[7] = (1 - f); p[8] = (1 - f);
    }
    if (c->isMT) {
      p[0] = f * f; p[1] = 0.0; p[2] = f * (1 - f); p[3] = 0; p[4] = 0; p[5] = 0;
      p[6] = (1 - f) * f; p[7] = 0; p[8] = (1 - f) * (1 - f);
    }
  } else {
    static const double trio[9] = {0.0, 0.24, 0.04, 0.24, 0.16, 0.08, 0.04, 0.08, 0.12};   /* :383-394 */
    memcpy(p, trio, sizeof(trio));
  }
}

/* SetParentPrior_denovo / SetParentPriorSingleTrio_denovo, :370-420 */
static void set_parent_prior_denovo(pmo_ctx *c, double f) {
  double *p = SC(c)->parentPrior;
  if (c->ped.n_fam > 1 || f == 1.0) {
    p[0] = (f * f) * (f * f);
    p[1] = f * f * f * (1 - f) * 2;
    p[2] = f * f * (1 - f) * (1 - f);
    p[3] = f * (1 - f) * 2 * f * f;
    p[4] = f * (1 - f) * 2 * f * (1 - f) * 2;
    p[5] = f * (1 - f) * 2 * (1 - f) * (1 - f);
    p[6] = (1 - f) * (1 - f) * f * f;
    p[7] = (1 - f) * (1 - f) * f * (1 - f) * 2;
    p[8] = (1 - f) * (1 - f) * (1 - f) * (1 - f);
  } else {
    static const double trio[9] = {0.0, 0.24, 0.04, 0.24, 0.16, 0.08, 0.04, 0.08, 0.12};
    memcpy(p, trio, sizeof(trio));
  }
}

/* ---------------- nuclear family closed form ---------------- */
static void geno_lk(const pmo_ctx *c, const lkobj *o, int person, double *l11, double *l12, double *l22) {
  *l11 = pen(c, person, o->g11); *l12 = pen(c, person, o->g12); *l22 = pen(c, person, o->g22);   /* :1633-1648 */
}

/* likelihoodONEKid, :1202-1264 (uses the object's member `sex`, quirk kept) */
static double one_kid(const pmo_ctx *c, int sex, int k, double l11, double l12, double l22) {
  const int X = c->isX, Y = c->isY, MT = c->isMT;
  switch (k) {
    case 0: return (Y && sex == FEMALE) ? 1.0 : l11;
    case 1: if (X) return sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l11 + l12);
            if (Y) return sex == MALE ? l11 : 1.0;
            if (MT) return 0.5 * (l11 + l22);
            return 0.5 * (l11 + l12);
    case 2: if (X) return sex == MALE ? l22 : l12;
            if (Y) return sex == MALE ? l11 : 1.0;
            if (MT) return l22;
            return l12;
    case 3: if (X || Y || MT) return 0.0; return 0.5 * (l11 + l12);
    case 4: if (X || Y || MT) return 0.0; return 0.25 * l11 + 0.5 * l12 + 0.25 * l22;
    case 5: if (X || Y || MT) return 0.0; return 0.5 * (l12 + l22);
    case 6: if (X) return sex == MALE ? l11 : l12;
            if (Y) return sex == MALE ? l22 : 1.0;
            if (MT) return l11;
            return l12;
    case 7: if (X) return sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l12 + l22);
            if (Y) return sex == MALE ? l22 : 1.0;
            if (MT) return 0.5 * (l11 + l22);
            return 0.5 * (l12 + l22);
    default: return (Y && sex == FEMALE) ? 1.0 : l22;
  }
}

/* CalcDenovoMutLk, :1553-1562 */
static double denovo_mut_lk(const pmo_ctx *c, int person, int x, int y) {
  double lk = 0.0; int idx = GI(x, y);
  for (int i = 0; i < 10; i++) lk += c->M[idx][i] * pen(c, person, i);
  return lk;
}

/* likelihoodONEKid_denovo, :1266-1296 */
static double one_kid_denovo(const pmo_ctx *c, const lkobj *o, int person, int k) {
  int a1 = o->a1, a2 = o->a2;
  switch (k) {
    case 0: return denovo_mut_lk(c, person, a1, a1);
    case 1: return 0.5 * (denovo_mut_lk(c, person, a1, a1) + denovo_mut_lk(c, person, a1, a2));
    case 2: return denovo_mut_lk(c, person, a1, a2);
    case 3: return 0.5 * (denovo_mut_lk(c, person, a1, a1) + denovo_mut_lk(c, person, a1, a2));
    case 4: return 0.25 * denovo_mut_lk(c, person, a1, a1) + 0.5 * denovo_mut_lk(c, person, a1, a2) + 0.25 * denovo_mut_lk(c, person, a2, a2);
    case 5: return 0.5 * (denovo_mut_lk(c, person, a1, a2) + denovo_mut_lk(c, person, a2, a2));
    case 6: return denovo_mut_lk(c, person, a1, a2);
    case 7: return 0.5 * (denovo_mut_lk(c, person, a1, a2) + denovo_mut_lk(c, person, a2, a2));
    default: return denovo_mut_lk(c, person, a2, a2);
  }
}

/* CalcParentMarginal (:1041-1084) and CalcParentMarginal_denovo (:1086-1132) */
static void parent_marginal(pmo_ctx *c, const lkobj *o, int f, double freq, int denovo) {
  int p0 = c->fam_start[f], n = fam_count(c, f);
  double F11, F12, F22, M11, M12, M22;
  geno_lk(c, o, p0, &F11, &F12, &F22);
  geno_lk(c, o, p0 + 1, &M11, &M12, &M22);
  if (!denovo) {
    if (c->isX) F12 = 0.0;
    if (c->isY) { M11 = M12 = M22 = 1.0; F12 = 0.0; }
    if (c->isMT) F12 = M12 = 0.0;
  }
  double lF[3] = {F11, F12, F22}, lM[3] = {M11, M12, M22};
  struct pmo_scratch *w = SC(c);
  for (int a = 0; a < 3; a++) for (int b = 0; b < 3; b++) w->parentGLF[3 * a + b] = lF[a] * lM[b];
  if (!denovo) set_parent_prior(c, o, freq);
  else set_parent_prior_denovo(c, freq);
  for (int k = 0; k < 9; k++) {
    double kids = 1.0;   /* likelihoodKids(_denovo), :1184-1198 / :1299-1312 */
    for (int j = 2; j < n; j++) {
      double t;
      if (!denovo) { double l11, l12, l22; geno_lk(c, o, p0 + j, &l11, &l12, &l22); t = one_kid(c, o->sex, k, l11, l12, l22); }
      else t = one_kid_denovo(c, o, p0 + j, k);
      kids *= t;
    }
    double cond = kids * w->parentGLF[k];
    w->parentMarginal[k] = cond * w->parentPrior[k];
  }
}

/* lkSinglePerson, :987-1004 */
static double single_person(const pmo_ctx *c, const lkobj *o, int person, double f) {
  double l11, l12, l22, pr[3];
  geno_lk(c, o, person, &l11, &l12, &l22);
  pr[0] = f * f; pr[1] = f * (1 - f) * 2; pr[2] = (1 - f) * (1 - f);
  int sx = c->sex[person];
  if (c->isX) { if (sx == MALE) { l12 = 0; pr[0] = f; pr[1] = 0; pr[2] = 1 - f; } }
  if (c->isY) { if (sx == MALE) { l12 = 0; pr[0] = f; pr[1] = 0; pr[2] = 1 - f; } else return 1.0; }
  if (c->isMT) { l12 = 0; pr[0] = f; pr[1] = 0; pr[2] = 1 - f; }
  double sum = 0.0;
  sum = sum + l11 * pr[0] + l12 * pr[1] + l22 * pr[2];
  return sum;
}

/* lkSingleFam / lkSingleFam_denovo, :941-975 */
static double lk_single_fam(pmo_ctx *c, const lkobj *o, int f, double freq, int denovo) {
  if (fam_allfounders(c, f)) {
    double lk = 1.0;
    for (int j = 0; j < fam_founders(c, f); j++) lk *= single_person(c, o, c->fam_start[f] + j, freq);
    return lk;
  }
  parent_marginal(c, o, f, freq, denovo);
  double sum = 0.0;
  const double *pm = SC(c)->parentMarginal;
  for (int k = 0; k < 9; k++) sum += pm[k];
  return sum;
}

/* ---------------- Elston-Stewart peeling ---------------- */
/* GetTransmissionProb_BA, FamilyLikelihoodES.cpp:1059-1075 */
static double tba(const pmo_ctx *c, int i, int j, int k, int child_sex) {
  double t = c->TBA[0][i][j][k];
  if (c->isX) t = (child_sex == MALE) ? c->TBA[2][i][j][k] : c->TBA[1][i][j][k];
  if (c->isY) t = (child_sex == MALE) ? c->TBA[3][i][j][k] : 1.0;
  if (c->isMT) t = c->TBA[4][i][j][k];
  return t;
}

static double *find_mp(pmo_ctx *c, int a, int b, int create) {
  struct pmo_scratch *w = SC(c);
  for (int i = 0; i < w->nmp; i++) if (w->mpkey[i][0] == a && w->mpkey[i][1] == b) return &w->mp[i][0][0];
  if (!create) return NULL;
  int i = w->nmp++;   /* SetMarriagePartials, :1400-1415: all ones */
  w->mpkey[i][0] = a; w->mpkey[i][1] = b;
  for (int x = 0; x < 10; x++) for (int y = 0; y < 10; y++) w->mp[i][x][y] = 1.0;
  return &w->mp[i][0][0];
}

/* One ES likelihood of family f.  ns = 3 (bi-allelic, CalcSingleFamLikelihood_BA, FamilyLikelihoodSeq.cpp:256-266)
 * or 10 (de novo, CalcSingleFamLikelihood_denovo, :269-279).  zero_person/zero_geno implement
 * FillZeroPenetrance (FamilyLikelihoodSeq.cpp:327-356): person zero_person keeps only genotype zero_geno. */
static double es_likelihood(pmo_ctx *c, const lkobj *o, int f, double freq, int ns, int zero_person, int zero_geno) {
  const int p0 = c->fam_start[f], n = fam_count(c, f), nf = c->fam_founders[f];
  const int gidx[3] = {o->g11, o->g12, o->g22};
  double *P = SC(c)->partials;
  /* penetrance with FillZeroPenetrance applied */
#define PEN(i, g) ((zero_person == (i) && (g) != zero_geno) ? 0.0 : pen(c, p0 + (i), (g)))
  for (int i = 0; i < n; i++) {
    int sx = c->sex[p0 + i];
    if (ns == 3) {
      /* SetFounderPriors_BA :666-687 + InitializePartials_BA :1449-1465 */
      double pr[3];
      if (i < nf) {
        pr[0] = freq * freq; pr[1] = 2 * freq * (1 - freq); pr[2] = (1 - freq) * (1 - freq);
        if (c->isX) if (sx == MALE) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; }
        if (c->isY) { if (sx == MALE) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; } else { pr[0] = 1; pr[1] = 1; pr[2] = 1; } }
        if (c->isMT) { pr[0] = freq; pr[1] = 0; pr[2] = 1 - freq; }
      }
      for (int j = 0; j < 3; j++) {
        if (c->is_founder[p0 + i]) P[i * 10 + j] = (c->isY && sx == FEMALE) ? 1.0 : pr[j] * PEN(i, gidx[j]);
        else P[i * 10 + j] = (c->isY && sx == FEMALE) ? 1.0 : PEN(i, gidx[j]);
      }
    } else {
      /* SetFounderPriors :643-664 + InitializePartials :1434-1446 */
      double pr[10];
      if (i < nf) {
        for (int j = 0; j < 10; j++) pr[j] = 0.0;
        pr[gidx[0]] = freq * freq; pr[gidx[1]] = 2 * freq * (1 - freq); pr[gidx[2]] = (1 - freq) * (1 - freq);
        if (c->isX) if (sx == MALE) { pr[gidx[0]] = freq; pr[gidx[1]] = 0; pr[gidx[2]] = 1 - freq; }
        if (c->isY) { if (sx == MALE) { pr[gidx[0]] = freq; pr[gidx[1]] = 0; pr[gidx[2]] = 1 - freq; } else { pr[gidx[0]] = 1; pr[gidx[1]] = 1; pr[gidx[2]] = 1; } }
        if (c->isMT) { pr[gidx[0]] = freq; pr[gidx[1]] = 0; pr[gidx[2]] = 1 - freq; }
      }
      for (int j = 0; j < 10; j++)
        P[i * 10 + j] = c->is_founder[p0 + i] ? pr[j] * PEN(i, j) : PEN(i, j);
    }
  }
#undef PEN
  SC(c)->nmp = 0;
  const pm_peel_step *st = c->steps + c->peel_start[f];
  const int nst = c->peel_start[f + 1] - c->peel_start[f];
  for (int s = 0; s < nst; s++) {
    const pm_peel_step *S = &st[s];
    if (S->type == 1) {   /* peelOffspring2Parents_BA :1105-1130 / _denovo :1289-1310 */
      int off = S->from0;
      double *mp = find_mp(c, S->to0, S->to1, 1);
      for (int i = 0; i < ns; i++) for (int j = 0; j < ns; j++) {
        double sum = 0;
        for (int k = 0; k < ns; k++) {
          double t = (ns == 3) ? tba(c, i, j, k, c->sex[p0 + off]) : c->T10dn[i][j][k];
          sum += t * P[off * 10 + k];
        }
        mp[i * 10 + j] *= sum;
      }
    } else if (S->type == 2) {   /* peelSpouse2Spouse_BA :1182-1230 / _denovo :1312-1356 */
      int sf = S->from0, stt = S->to0, a, b, fa2mo;
      if (c->sex[p0 + sf] == 2) { a = stt; b = sf; fa2mo = 0; } else { a = sf; b = stt; fa2mo = 1; }
      double *mp = find_mp(c, a, b, 0);
      for (int i = 0; i < ns; i++) {
        double sum = 0.0;
        if (mp == NULL) for (int j = 0; j < ns; j++) sum += P[sf * 10 + j];
        else if (fa2mo) for (int j = 0; j < ns; j++) sum += P[sf * 10 + j] * mp[j * 10 + i];
        else for (int j = 0; j < ns; j++) sum += P[sf * 10 + j] * mp[i * 10 + j];
        P[stt * 10 + i] *= sum;
      }
    } else {   /* peelParents2Offspring_BA :1260-1286 / _denovo :1358-1395 */
      int fa = S->from0, mo = S->from1, off = S->to0;
      double *mp = find_mp(c, fa, mo, 0);
      for (int k = 0; k < ns; k++) {
        double sum = 0.0;
        for (int i = 0; i < ns; i++) for (int j = 0; j < ns; j++) {
          double t;
          if (ns == 3) t = tba(c, i, j, k, c->sex[p0 + off]);
          else t = (mp == NULL) ? c->T10dn[i][j][k] : c->T10[i][j][k];   /* quirk: plain transmission with partials (:1391) */
          if (mp == NULL) sum += P[fa * 10 + i] * P[mo * 10 + j] * t;
          else sum += P[fa * 10 + i] * mp[i * 10 + j] * P[mo * 10 + j] * t;
        }
        P[off * 10 + k] *= sum;
      }
    }
  }
  int fin = st[nst - 1].to0;   /* CalculateLikelihood_BA :1013-1032 */
  double lk = 0.0;
  for (int i = 0; i < ns; i++) lk += P[fin * 10 + i];
  return lk;
}

/* ---------------- objective ---------------- */
/* FamilyLikelihoodSeq::CalcAllFamLogLikelihood, FamilyLikelihoodSeq.cpp:222-240 (serial family order) */
static double all_fam_loglik(pmo_ctx *c, lkobj *o, double freq) {
  double loglk = 0.0;
  /* the reference's family loop is an `omp parallel for reduction(+:loglk)` (:225): inside the configuration sections
   * it is an inactive nested region (serial, in family order); only the de novo LR re-optimisation outside them
   * (main.cpp:569-572) runs it on several threads, with a thread-count-dependent summation order */
#pragma omp parallel for reduction(+:loglk)
  for (int f = 0; f < c->ped.n_fam; f++) {
    if (fam_nuclear(c, f) || fam_allfounders(c, f))
      loglk += log10(lk_single_fam(c, o, f, freq, c->denovo));
    else
      loglk += log10(es_likelihood(c, o, f, freq, c->denovo ? 10 : 3, -1, -1));
  }
  return loglk;
}

static double vcf_all_fam_loglik(pmo_ctx *c, lkobj *o, double freq);
static double objf(pmo_ctx *c, lkobj *o, double x) {   /* :39-42; FamilyLikelihoodSeq_VCF.cpp:31-34 */
  o->evals++;
  return c->vcf_objective ? -vcf_all_fam_loglik(c, o, x) : -all_fam_loglik(c, o, x);
}

/* OptimizeFrequency (NucFamGenotypeLikelihood.cpp:432-444) + ScalarMinimizer::Brent (core/MathGold.cpp:81-177) */
static int optimize(pmo_ctx *c, lkobj *o) {
  double a = 0.0001, fa = objf(c, o, a);
  double b = 0.9999, fb = objf(c, o, b);
  double cc = 0.5, fc = objf(c, o, cc);
  double tol = c->par.precision, temp;
  if (a > cc) { temp = a; a = cc; cc = temp; temp = fa; fa = fc; fc = temp; }
  double min = b, fmin = fb, w = b, v = b, fw = fb, fv = fb, delta = 0.0, u, fu, d = 0.0;
  (void)fa; (void)fc;
  for (int iter = 1; iter <= c->itmax; iter++) {
    double middle = 0.5 * (a + cc);
    double tol1 = tol * fabs(min) + ZEPS;
    double tol2 = 2.0 * tol1;
    if (fabs(min - middle) <= (tol2 - 0.5 * (cc - a))) { o->min = min; o->fmin = fmin; return 0; }
    if (fabs(delta) > tol1) {
      double r = (min - w) * (fmin - fv);
      double q = (min - v) * (fmin - fw);
      double p = (min - v) * q - (min - w) * r;
      q = 2.0 * (q - r);
      if (q > 0.0) p = -p;
      q = fabs(q);
      temp = delta; delta = d;
      if (fabs(p) >= fabs(0.5 * q * temp) || p <= q * (a - min) || p >= q * (cc - min)) {
        delta = min >= middle ? a - min : cc - min;
        d = CGOLD * delta;
      } else {
        d = p / q;
        u = min + d;
        if (u - a < tol2 || cc - u < tol2) d = sign_(tol1, middle - min);
      }
    } else {
      delta = min >= middle ? a - min : cc - min;
      d = CGOLD * delta;
    }
    u = fabs(d) >= tol1 ? min + d : min + sign_(tol1, d);
    fu = objf(c, o, u);
    if (fu <= fmin) {
      if (u >= min) a = min; else cc = min;
      v = w; w = min; min = u;
      fv = fw; fw = fmin; fmin = fu;
    } else {
      if (u < min) a = u; else cc = u;
      if (fu <= fw || w == min) { v = w; w = u; fv = fw; fw = fu; }
      else if (fu <= fv || v == min || v == w) { v = u; fv = fu; }
    }
  }
  o->min = min; o->fmin = fmin;
  return PM_EBRENT;   /* numerror("ScalarMinimizer::Brent got stuck") */
}

static int g_brent_err;
/* FamilyLikelihoodSeq::PolymorphismLogLikelihood, FamilyLikelihoodSeq.cpp:91-104 */
static double poly_loglik(pmo_ctx *c, lkobj *o, int a1, int a2) {
  set_alleles(c, o, a1, a2);
  if (c->ped.n_fam > 1 || (c->ped.n_fam == 1 && !fam_nuclear(c, 0))) {
    if (optimize(c, o) != 0) {
#pragma omp atomic write
      g_brent_err = 1;
    }
    return -o->fmin;
  }
  o->evals++;
  return all_fam_loglik(c, o, 0.5);
}

/* MonomorphismLogLikelihood, NucFamGenotypeLikelihood.cpp:502-517 */
static double mono_loglik(const pmo_ctx *c) {
  double l = 0.0; int h = GI(c->refBase, c->refBase);
  for (int p = 0; p < c->ped.n_person; p++) l += -(double)(c->pl[p * 10 + h]) / 10;
  return l;
}

/* ---------------- model selection ---------------- */
/* CalcVarPosterior / CalcMaxLogLkIdx / CalcMaxLogLkAlt / CalcPolyQual, NucFamGenotypeLikelihood.cpp:1650-1749 */
static int var_posterior(pmo_ctx *c, const double *varllk, int n, double *vpp, double *qual) {
  int idx = 0; double max = varllk[0];
  for (int i = 0; i < n; i++) if (max < varllk[i]) { max = varllk[i]; idx = i; }
  double sum = 0.0;
  for (int i = 0; i < n; i++) sum += exp10(varllk[i] - varllk[idx]);
  *vpp = 1 / sum;
  int r = c->refBase, ts = poly_ts(r), tv1 = poly_tv1(r), tv2 = poly_tv2(r), a1 = 0, a2 = 0;
  if (idx == 0) {
    int k = 1; double m = varllk[1];
    for (int i = 1; i < 4; i++) if (m < varllk[i]) { m = varllk[i]; k = i; }
    a1 = r; a2 = (k == 1) ? ts : (k == 2) ? tv1 : tv2;
  } else if (idx == 1) { a1 = r; a2 = ts; }
  else if (idx == 2) { a1 = r; a2 = tv1; }
  else if (idx == 3) { a1 = r; a2 = tv2; }
  else if (idx == 4) { a1 = ts; a2 = tv1; }
  else if (idx == 5) { a1 = ts; a2 = tv2; }
  else { a1 = tv1; a2 = tv2; }
  set_alleles(c, &c->lk[0], a1, a2);
  *qual = (*vpp > 0.9999999999) ? 100 : -10 * log10(1 - *vpp);
  return idx;
}

/* ---------------- posteriors ---------------- */
static int best3(double p11, double p12, double p22) {   /* GetBestGenoIdx, :1564-1571 */
  int b = 0; double m = p11;
  if (p12 > m) { m = p12; b = 1; }
  if (p22 > m) { m = p22; b = 2; }
  return b;
}
/* which labeller GetBestGenoLabel_vcfv4 (:1590-1608) picks for a person given the object's member sex */
static int8_t vcf_label(const pmo_ctx *c, int membersex) {
  if (c->isY || c->isMT) return PM_LBL_VCF_HAPLOID;
  if (c->isX && membersex == MALE) return PM_LBL_VCF_HAPLOID;
  return PM_LBL_VCF_DIPLOID;
}

static void set3(pmo_ctx *c, int p, double a, double b, double d) { c->postv[p * 10 + 0] = a; c->postv[p * 10 + 1] = b; c->postv[p * 10 + 2] = d; }

/* CalcPostProb_SinglePerson, :754-795 */
static void post_single_person(pmo_ctx *c, lkobj *o, int p, double f) {
  double l11, l12, l22, pr[3];
  pr[0] = f * f; pr[1] = f * (1 - f) * 2; pr[2] = (1 - f) * (1 - f);
  geno_lk(c, o, p, &l11, &l12, &l22);
  int sx = c->sex[p];
  if (c->isX) { if (sx == MALE) { pr[0] = f; pr[1] = 0.; pr[2] = 1 - f; } else { pr[0] = f * f; pr[1] = 2 * f * (1 - f); pr[2] = (1 - f) * (1 - f); } }
  if (c->isY) { if (sx == MALE) { pr[0] = f; pr[1] = 0.; pr[2] = 1 - f; } else { pr[0] = pr[1] = pr[2] = 1.0; } }
  if (c->isMT) { pr[0] = f; pr[1] = 0; pr[2] = 1 - f; }
  double m11 = l11 * pr[0], m12 = l12 * pr[1], m22 = l22 * pr[2];
  double sum = m11 + m12 + m22;
  if (sum == 0) set3(c, p, 0, 0, 0);   /* 1/3 is integer division */
  else set3(c, p, m11 / sum, m12 / sum, m22 / sum);
  if (c->isY && sx == FEMALE) set3(c, p, 0.0, 0.0, 0.0);
  c->best[p] = best3(m11, m12, m22);
  c->label[p] = (c->isY && sx == FEMALE) ? PM_LBL_DOT : vcf_label(c, o->sex);
  c->dosage[p] = c->postv[p * 10 + 1] + c->postv[p * 10 + 2] * 2;
}

/* likelihoodKidGenotype, :1334-1443: returns g11,g12,g22 for kid `kid` under parental config k */
static void kid_geno(pmo_ctx *c, lkobj *o, int f, int kid, int k, double *g) {
  const int p0 = c->fam_start[f], n = fam_count(c, f), X = c->isX, Y = c->isY, MT = c->isMT;
  double G11 = 1.0, G12 = 1.0, G22 = 1.0, lk = 0.0, q11 = 0, q12 = 0, q22 = 0;
  for (int i = 2; i < n; i++) {
    double l11, l12, l22;
    geno_lk(c, o, p0 + i, &l11, &l12, &l22);
    int sex = c->sex[p0 + i];
    switch (k) {
      case 0: lk = l11; q11 = l11; q12 = q22 = 0; break;
      case 1:
        if (X) { lk = sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l11 + l12);
                 if (sex == MALE) { q11 = 0.5 * l11; q12 = 0.0; q22 = 0.5 * l22; } else { q11 = 0.5 * l11; q12 = 0.5 * l12; q22 = 0; } }
        else if (Y) { lk = sex == MALE ? l11 : 1.0; if (sex == MALE) { q11 = l11; q12 = q22 = 0.0; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { lk = 0.5 * (l11 + l22); q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; }
        else { lk = 0.5 * (l11 + l12); q11 = l11 * 0.5; q12 = l12 * 0.5; q22 = 0; }
        break;
      case 2:
        if (X) { lk = sex == MALE ? l22 : l12; if (sex == MALE) { q11 = q12 = 0; q22 = l22; } else { q11 = q22 = 0; q12 = l12; } }
        else if (Y) { lk = sex == MALE ? l11 : 1.0; if (sex == MALE) { q11 = l11; q12 = q22 = 0; } else { q11 = q12 = q22 = 0.; } }
        else if (MT) { lk = l22; q11 = q12 = 0; q22 = l22; }
        else { lk = l12; q11 = 0; q12 = l12; q22 = 0; }
        break;
      case 3:
        if (X || Y || MT) { lk = 0.0; q11 = q12 = q22 = 0.0; }
        else { lk = 0.5 * (l11 + l12); q11 = l11 * 0.5; q12 = l12 * 0.5; q22 = 0; }
        break;
      case 4:
        if (X || Y || MT) { lk = 0.0; q11 = q12 = q22 = 0.0; }
        else { lk = 0.25 * l11 + 0.5 * l12 + 0.25 * l22; q11 = l11 * 0.25; q12 = l12 * 0.5; q22 = l22 * 0.25; }
        break;
      case 5:
        if (X || Y || MT) { lk = 0.0; q11 = q12 = q22 = 0.0; }
        else { lk = 0.5 * (l12 + l22); q11 = 0; q12 = l12 * 0.5; q22 = l22 * 0.5; }
        break;
      case 6:
        if (X) { lk = sex == MALE ? l11 : l12; if (sex == MALE) { q11 = l11; q12 = q22 = 0.0; } else { q11 = q22 = 0.0; q12 = l12; } }
        else if (Y) { lk = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { lk = l11; q11 = l11; q12 = q22 = 0.0; }
        else { lk = l12; q11 = 0; q12 = l12; q22 = 0; }
        break;
      case 7:
        if (X) { lk = sex == MALE ? 0.5 * (l11 + l22) : 0.5 * (l12 + l22);
                 if (sex == MALE) { q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; } else { q11 = 0.0; q12 = 0.5 * l12; q22 = 0.5 * l22; } }
        else if (Y) { lk = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q12 = q22 = 0.0; } }
        else if (MT) { lk = 0.5 * (l11 + l22); q11 = 0.5 * l11; q22 = 0.5 * l22; q12 = 0.0; }
        else { lk = 0.5 * (l12 + l22); q11 = 0; q12 = l12 * 0.5; q22 = l22 * 0.5; }
        break;
      default:   /* 22 x 22: if/if/if-else chain, :1416-1422 -- for X and Y the trailing else overrides */
        if (X) { lk = l22; q11 = 0.0; q22 = l22; }
        if (Y) { lk = sex == MALE ? l22 : 1.0; if (sex == MALE) { q11 = q12 = 0.0; q22 = l22; } else { q11 = q22 = q12 = 0.0; } }
        if (MT) { lk = l22; q11 = q12 = 0.0; q22 = l22; }
        else { lk = l22; q11 = 0; q12 = 0; q22 = l22; }
        break;
    }
    if (i != kid) { G11 *= lk; G12 *= lk; G22 *= lk; }
    else { G11 *= q11; G12 *= q12; G22 *= q22; }
  }
  g[0] = G11; g[1] = G12; g[2] = G22;
}

/* GetJointGenoLk_denovo, :1480-1551 */
static void joint_geno_denovo(pmo_ctx *c, lkobj *o, int person, int k, double *out) {
  int i1 = GI(o->a1, o->a1), i2 = GI(o->a1, o->a2), i3 = GI(o->a2, o->a2);
  for (int i = 0; i < 10; i++) {
    double m, p = pen(c, person, i);
    switch (k) {
      case 0: m = c->M[i1][i]; break;
      case 1: case 3: m = 0.5 * c->M[i1][i] + 0.5 * c->M[i2][i]; break;
      case 2: case 6: m = c->M[i2][i]; break;
      case 4: m = 0.25 * c->M[i1][i] + 0.5 * c->M[i2][i] + 0.25 * c->M[i3][i]; break;
      case 5: case 7: m = 0.5 * c->M[i2][i] + 0.5 * c->M[i3][i]; break;
      default: m = c->M[i3][i]; break;
    }
    out[i] = m * p;
  }
}

/* CalcPostProb_SingleNucFam (:590-669) and _denovo (:671-752) */
static void post_nuc(pmo_ctx *c, lkobj *o, int f, double freq, int denovo) {
  const int p0 = c->fam_start[f], n = fam_count(c, f);
  if (n <= fam_founders(c, f)) {
    for (int j = 0; j < fam_founders(c, f); j++) {
      if (!denovo) o->sex = c->sex[p0 + j];
      post_single_person(c, o, p0 + j, freq);
    }
    return;
  }
  parent_marginal(c, o, f, freq, denovo);
  const double *m = SC(c)->parentMarginal;
  for (int j = 0; j < n; j++) {
    int p = p0 + j;
    if (!denovo) o->sex = c->sex[p];
    if (j < 2) {
      double q11, q12, q22;
      if (j == 0) { q11 = m[0] + m[1] + m[2]; q12 = m[3] + m[4] + m[5]; q22 = m[6] + m[7] + m[8]; }
      else { q11 = m[0] + m[3] + m[6]; q12 = m[1] + m[4] + m[7]; q22 = m[2] + m[5] + m[8]; }
      double sum = q11 + q12 + q22;
      if (sum == 0) set3(c, p, 0, 0, 0);
      else set3(c, p, q11 / sum, q12 / sum, q22 / sum);
      c->best[p] = best3(q11, q12, q22);
      if (!denovo) c->label[p] = (c->isY && c->sex[p] == FEMALE) ? PM_LBL_DOT : vcf_label(c, o->sex);
      else c->label[p] = PM_LBL_ALLELES;
      c->dosage[p] = c->postv[p * 10 + 1] + c->postv[p * 10 + 2] * 2;
    } else if (!denovo) {
      /* KidJointGenoLikelihood :798-835 + JointGenoLk::CalcPost (src/PedigreeGLF.cpp:13-22) */
      double J[9][3];
      for (int k = 0; k < 9; k++) {
        kid_geno(c, o, f, j, k, J[k]);
        double w = SC(c)->parentGLF[k] * SC(c)->parentPrior[k];
        J[k][0] *= w; J[k][1] *= w; J[k][2] *= w;
      }
      double g[3];
      for (int t = 0; t < 3; t++) {
        g[t] = J[0][t] + J[1][t] + J[2][t] + J[3][t] + J[4][t] + J[5][t] + J[6][t] + J[7][t] + J[8][t];
      }
      double sum = g[0] + g[1] + g[2];
      if (sum == 0.0) set3(c, p, 0, 0, 0);
      else set3(c, p, g[0] / sum, g[1] / sum, g[2] / sum);
      c->best[p] = best3(c->postv[p * 10], c->postv[p * 10 + 1], c->postv[p * 10 + 2]);
      c->label[p] = (c->isY && c->sex[p] == FEMALE) ? PM_LBL_DOT : vcf_label(c, o->sex);
      c->dosage[p] = c->postv[p * 10 + 1] + c->postv[p * 10 + 2] * 2;
    } else {
      /* KidJointGenoLikelihood_denovo :838-868, likelihoodKidGenotype_denovo :1446-1478 */
      double J[9][10];
      for (int k = 0; k < 9; k++) {
        for (int t = 0; t < 10; t++) J[k][t] = 1.0;
        for (int i = 2; i < n; i++) {
          if (i != j) { double lk = one_kid_denovo(c, o, p0 + i, k); for (int t = 0; t < 10; t++) J[k][t] *= lk; }
          else { double jt[10]; joint_geno_denovo(c, o, p0 + i, k, jt); for (int t = 0; t < 10; t++) J[k][t] *= jt[t]; }
        }
        double w = SC(c)->parentGLF[k] * SC(c)->parentPrior[k];
        for (int t = 0; t < 10; t++) J[k][t] *= w;
      }
      double g[10], sum = 0.0;
      for (int t = 0; t < 10; t++) g[t] = 0.0;
      for (int t = 0; t < 10; t++) for (int k = 0; k < 9; k++) g[t] += J[k][t];
      for (int t = 0; t < 10; t++) sum += g[t];   /* JointGenoLk_denovo::CalcPost, src/PedigreeGLF.cpp:38-51 */
      for (int t = 0; t < 10; t++) c->postv[p * 10 + t] = (sum == 0.0) ? 0.0 : g[t] / sum;
      double mx = 0.0; int b = 0;
      for (int t = 0; t < 10; t++) if (mx < c->postv[p * 10 + t]) { mx = c->postv[p * 10 + t]; b = t; }
      c->best[p] = b;
      c->label[p] = PM_LBL_GENO10;
      c->dosage[p] = 0.0;
    }
  }
}

/* CalcPostProb_SingleExtendedPed_BA (FamilyLikelihoodSeq.cpp:171-216) and _denovo (:140-169) */
static void post_ext(pmo_ctx *c, lkobj *o, int f, double freq, int denovo) {
  const int p0 = c->fam_start[f], n = fam_count(c, f);
  for (int j = 0; j < n; j++) {
    int p = p0 + j;
    if (!denovo) {
      o->sex = c->sex[p];
      if (c->isY && c->sex[p] == FEMALE) { c->best[p] = 0; c->label[p] = PM_LBL_DOT; set3(c, p, 0, 0, 0); c->dosage[p] = 0; continue; }
      double l11 = es_likelihood(c, o, f, freq, 3, j, o->g11);
      double l12 = es_likelihood(c, o, f, freq, 3, j, o->g12);
      double l22 = es_likelihood(c, o, f, freq, 3, j, o->g22);
      double sum = l11 + l12 + l22;
      if (sum == 0) set3(c, p, 0, 0, 0);
      else set3(c, p, l11 / sum, l12 / sum, l22 / sum);
      c->best[p] = best3(l11, l12, l22);
      c->label[p] = vcf_label(c, o->sex);
      c->dosage[p] = c->postv[p * 10 + 1] + c->postv[p * 10 + 2] * 2;
    } else {
      double lk[10], sum = 0.0;
      for (int k = 0; k < 10; k++) lk[k] = es_likelihood(c, o, f, freq, 10, j, k);
      for (int k = 0; k < 10; k++) sum += lk[k];
      for (int k = 0; k < 10; k++) c->postv[p * 10 + k] = (sum == 0) ? 0 : lk[k] / sum;
      int b = 0; double mx = 0.0;
      for (int k = 0; k < 10; k++) if (mx < lk[k]) { mx = lk[k]; b = k; }
      c->best[p] = b; c->label[p] = PM_LBL_GENO10;
      /* dosage is left stale by the reference (not printed by OutputVCF_denovo) */
      c->dosage[p] = 0.0;
    }
  }
}

/* FamilyLikelihoodSeq::CalcPostProb, FamilyLikelihoodSeq.cpp:74-89 */
static void calc_post_prob(pmo_ctx *c, double freq) {
  lkobj *o = &c->lk[0];
  for (int f = 0; f < c->ped.n_fam; f++) {
    if (fam_nuclear(c, f) || fam_allfounders(c, f)) post_nuc(c, o, f, freq, c->denovo);
    else post_ext(c, o, f, freq, c->denovo);
  }
  c->any_postprob = 1;
}

/* CalculateAB, NucFamGenotypeLikelihood.cpp:1006-1039 */
static double calc_ab(pmo_ctx *c, const lkobj *o, double freq) {
  double A = 0.0, B = 0.0, p11 = freq * freq, p12 = 2 * freq * (1 - freq), p22 = (1 - freq) * (1 - freq);
  for (int p = 0; p < c->ped.n_person; p++) {
    int depth = (int)(c->dm[p] & 0xFFFFFF);
    double l11, l12, l22;
    geno_lk(c, o, p, &l11, &l12, &l22);
    int k11 = c->pl[p * 10 + o->g11], k12 = c->pl[p * 10 + o->g12], k22 = c->pl[p * 10 + o->g22];
    double PHet = (p12 * l12) / (p11 * l11 + p12 * l12 + p22 * l22);
    if (PHet > 1e-05 && depth > 0) {
      int scale = k22 + k11 - 2 * k12 + 6 * depth;
      int minimum = abs(k22 - k11);
      if (scale < 4) scale = 4;
      if (scale < minimum) scale = minimum;
      int nRef = 0.5 * depth * (1 + (k22 - k11) / (scale + 1e-30));
      A += PHet * nRef;
      B += PHet * depth;
    }
  }
  return (0.05 + A) / (0.1 + B);
}

static void fill_calls(pmo_ctx *c, pm_geno_call *calls) {
  for (int p = 0; p < c->ped.n_person; p++) {
    int b = c->best[p];
    double pb = c->postv[p * 10 + b];
    int gq = (pb > 0.9999999999) ? 100 : (int)(-10. * log10(1. - pb) + 0.5);   /* OutputVCF :1818-1820 */
    calls[p].dosage = c->dosage[p];
    calls[p].best = (int16_t)b;
    calls[p].gq = (int16_t)gq;
    calls[p].label = c->label[p];
    calls[p]._pad[0] = calls[p]._pad[1] = calls[p]._pad[2] = 0;
  }
}

/* ---------------- --in_vcf path (FamilyLikelihoodSeq_VCF, PedVCF) ---------------- */
/* Family kinds as FamilyLikelihoodSeq_VCF::CalcAllFamLogLikelihood / CalcPostProb route them
 * (src/FamilyLikelihoodSeq_VCF.cpp:93-109, :142-154): all-founder, nuclear closed form (only for
 * nFam > 1 on autosomes), everything else Elston-Stewart BA peeling. */
static int vcf_closed_form(const pmo_ctx *c, int f) {
  return c->fam_kind[f] == PM_FAM_NUCLEAR && c->ped.n_fam > 1 && !c->isX && !c->isY && !c->isMT;
}

/* FamilyLikelihoodSeq_VCF::CalcAllFamLogLikelihood (:93-109) incl. CalcSingleFamLogLikelihood_Founders (:111-119) */
static double vcf_all_fam_loglik(pmo_ctx *c, lkobj *o, double freq) {
  double loglk = 0.0;
  for (int f = 0; f < c->ped.n_fam; f++) {
    const int p0 = c->fam_start[f], n = fam_count(c, f);
    if (n == c->fam_founders[f]) {
      double llk = 0.0;
      for (int j = 0; j < n; j++) llk += log10(single_person(c, o, p0 + j, freq));
      loglk += llk;
    } else if (vcf_closed_form(c, f)) {
      parent_marginal(c, o, f, freq, 0);   /* lkSingleFam :527-535; SetParentPrior since nFam > 1 */
      double sum = 0.0;
      for (int k = 0; k < 9; k++) sum += SC(c)->parentMarginal[k];
      loglk += log10(sum);
    } else {
      loglk += log10(es_likelihood(c, o, f, freq, 3, -1, -1));   /* CalcSingleFamLogLikelihood_BA */
    }
  }
  return loglk;
}

/* OptimizeFrequency + Brent over f = -CalcAllFamLogLikelihood (FamilyLikelihoodSeq_VCF::f :31-34) */
static int vcf_optimize(pmo_ctx *c, lkobj *o) {
  c->vcf_objective = 1;
  int rc = optimize(c, o);
  c->vcf_objective = 0;
  return rc;
}

/* FamilyLikelihoodSeq_VCF::CalcPostProb (:140-156) */
static void vcf_calc_post_prob(pmo_ctx *c, lkobj *o, double freq) {
  for (int f = 0; f < c->ped.n_fam; f++) {
    const int p0 = c->fam_start[f], n = fam_count(c, f);
    if (n == c->fam_founders[f]) {   /* CalcPostProb_SingleFam_BA_Founders_VCF :158-165 */
      for (int j = 0; j < n; j++) { o->sex = c->sex[p0 + j]; post_single_person(c, o, p0 + j, freq); }
    } else if (vcf_closed_form(c, f)) {
      post_nuc(c, o, f, freq, 0);    /* CalcPostProb_SingleNucFam :656-735 (same arithmetic as the GLF path) */
    } else {
      post_ext(c, o, f, freq, 0);    /* CalcPostProb_SingleExtendedPed_BA_VCF :207-262 */
    }
  }
}

/* One biallelic record with data of PedVCF::VarCallFromVCF (src/PedVCF.cpp:118-162): mono, one Brent,
 * posteriors at the minimiser.  QUAL/AF/AC/DP formatting stays with the caller (host). */
static int vcf_site(pmo_ctx *c, const uint8_t *pl, int32_t ref_alt, pm_site_result *R, pm_geno_call *calls) {
  const int a1 = ref_alt & 15, a2 = (ref_alt >> 4) & 15;
  if (a1 < 1 || a1 > 4 || a2 < 1 || a2 > 4 || a1 == a2) { R->status = PM_SITE_BAD_REF; return 0; }
  R->status = PM_SITE_CALLED;
  /* MonomorphismLogLikelihood (:74-83): loglk[homref] = -min(PL,255)/10, summed in family/person order */
  double mono = 0.0; const int h = GI(a1, a1);
  for (int p = 0; p < c->ped.n_person; p++) mono += -(double)(pl[p * 10 + h]) / 10;
  lkobj *o = &c->lk[1];
  o->evals = 0;
  set_alleles(c, o, a1, a2);
  if (vcf_optimize(c, o) != 0) return PM_EBRENT;
  R->n_cfg = 2; R->maxidx = 1;
  R->varllk[0] = mono; R->varllk[1] = -o->fmin;
  R->varfreq[0] = 1.0; R->varfreq[1] = o->min;
  R->evals[1] = (int32_t)o->evals;
  R->allele1 = a1; R->allele2 = a2; R->af = o->min; R->ab = 0.5; R->denovo_lr = -1;
  lkobj *o0 = &c->lk[0];
  set_alleles(c, o0, a1, a2);
  vcf_calc_post_prob(c, o0, o->min);
  R->emit = 1; R->call_row = 0;
  fill_calls(c, calls);
  return 0;
}

/* ---------------- public API ---------------- */
pmo_ctx *pmo_create(const pm_pedigree *ped, const pm_params *par) {
  pmo_ctx *c = (pmo_ctx *)calloc(1, sizeof(pmo_ctx));
  c->ped = *ped; c->par = *par;
  c->itmax = ITMAX;
  const char *eit = getenv("PM_TEST_ITMAX");
  if (eit && atoi(eit) > 0 && atoi(eit) < ITMAX) c->itmax = atoi(eit);
  int nf = ped->n_fam, np = ped->n_person, ns = ped->peel_start ? ped->peel_start[nf] : 0;
  c->fam_start = malloc(sizeof(int32_t) * (nf + 1)); memcpy(c->fam_start, ped->fam_start, sizeof(int32_t) * (nf + 1));
  c->fam_founders = malloc(sizeof(int32_t) * nf); memcpy(c->fam_founders, ped->fam_founders, sizeof(int32_t) * nf);
  c->fam_kind = malloc(sizeof(int32_t) * nf); memcpy(c->fam_kind, ped->fam_kind, sizeof(int32_t) * nf);
  c->peel_start = calloc(nf + 1, sizeof(int32_t));
  if (ped->peel_start) memcpy(c->peel_start, ped->peel_start, sizeof(int32_t) * (nf + 1));
  c->steps = malloc(sizeof(pm_peel_step) * (ns + 1));
  if (ns) memcpy(c->steps, ped->steps, sizeof(pm_peel_step) * ns);
  c->sex = malloc(np); memcpy(c->sex, ped->sex, np);
  c->is_founder = malloc(np); memcpy(c->is_founder, ped->is_founder, np);
  int maxfs = 1;
  for (int f = 0; f < nf; f++) if (c->fam_start[f + 1] - c->fam_start[f] > maxfs) maxfs = c->fam_start[f + 1] - c->fam_start[f];
  c->scr = calloc(PMO_MAXT, sizeof(struct pmo_scratch));
  for (int t = 0; t < PMO_MAXT; t++) c->scr[t].partials = malloc(sizeof(double) * 10 * maxfs);
  c->postv = calloc((size_t)np * 10, sizeof(double));
  c->best = calloc(np, sizeof(int)); c->label = calloc(np, 1); c->dosage = calloc(np, sizeof(double));
  c->denovo = par->denovo;
  build_tables(c);
  for (int r = 0; r < 7; r++) { c->lk[r].min = 0.0; c->lk[r].fmin = 0.0; }
  pmo_begin_section(c, PM_CHR_AUTO);
  return c;
}

void pmo_destroy(pmo_ctx *c) {
  if (!c) return;
  free(c->fam_start); free(c->fam_founders); free(c->fam_kind); free(c->peel_start); free(c->steps);
  free(c->sex); free(c->is_founder);
  for (int t = 0; t < PMO_MAXT; t++) free(c->scr[t].partials);
  free(c->scr); free(c->postv); free(c->best); free(c->label); free(c->dosage);
  free(c);
}

/* famlk[0] after CalcPostProb holds the last person's sex (calc_post_prob visits every person in order) */
void pmo_set_posterior_carry(pmo_ctx *c, int32_t seen) {
  c->any_postprob = seen != 0;
  c->lk[0].sex = seen ? c->sex[c->ped.n_person - 1] : 0;
}

void pmo_begin_section(pmo_ctx *c, int32_t chrom) {
  c->chrom = chrom; c->isX = chrom == PM_CHR_X; c->isY = chrom == PM_CHR_Y; c->isMT = chrom == PM_CHR_MT;
  c->prior = poly_prior(c);
  memset(&c->cnt, 0, sizeof(c->cnt));
}

double pmo_poly_prior(const pmo_ctx *c) { return c->prior; }
void pmo_counters(const pmo_ctx *c, pm_counters *out) { *out = c->cnt; }
const double *pmo_geno_mut_matrix(const pmo_ctx *c) { return &c->M[0][0]; }

double pmo_objective(pmo_ctx *c, const uint8_t *pl, int32_t a1, int32_t a2, double freq, int32_t denovo) {
  lkobj o; memset(&o, 0, sizeof(o));
  c->pl = pl; set_alleles(c, &o, a1, a2);
  int save = c->denovo; c->denovo = denovo;
  double r = -all_fam_loglik(c, &o, freq);
  c->denovo = save;
  return r;
}

double pmo_poly_loglik(pmo_ctx *c, const uint8_t *pl, int32_t a1, int32_t a2, int32_t denovo, double *min_out, int32_t *evals) {
  lkobj o; memset(&o, 0, sizeof(o));
  c->pl = pl;
  int save = c->denovo; c->denovo = denovo;
  double r = poly_loglik(c, &o, a1, a2);
  c->denovo = save;
  if (min_out) *min_out = o.min;
  if (evals) *evals = (int32_t)o.evals;
  return r;
}

/* One iteration of the site loop body, src/main.cpp:327-594. */
int pmo_site(pmo_ctx *c, const uint8_t *pl, const uint32_t *dm, int32_t refBase, pm_site_result *R, pm_geno_call *calls) {
  memset(R, 0, sizeof(*R));
  R->maxidx = -2; R->call_row = -1;
  c->pl = pl; c->dm = dm; c->refBase = refBase & 15;
  g_brent_err = 0;
  if (c->par.vcf_mode) return vcf_site(c, pl, refBase, R, calls);
  if (refBase < 1 || refBase > 4) { R->status = PM_SITE_BAD_REF; return 0; }
  c->cnt.ref_base_counts[refBase]++;
  /* CalcReadStats, NucFamGenotypeLikelihood.cpp:520-546 */
  int td = 0, nsd = 0; double mq = 0.0;
  for (int p = 0; p < c->ped.n_person; p++) {
    int d = (int)(dm[p] & 0xFFFFFF);
    td += d; mq += (double)(dm[p] >> 24);
    if (d > 0) nsd++;
  }
  double avgmq = 0., ps = 0.;
  if (nsd > 0) { avgmq = mq / (double)nsd; ps = (double)nsd / (double)c->ped.n_person; }
  R->total_depth = td; R->num_samp_with_data = nsd; R->avg_map_qual = avgmq; R->perc_samp_with_data = ps;
  const pm_params *P = &c->par;
  if (td < P->min_total_depth) { c->cnt.min_total_depth_filter++; R->status = PM_SITE_MIN_DEPTH; return 0; }
  if (P->max_total_depth > 0 && td > P->max_total_depth) { c->cnt.max_total_depth_filter++; R->status = PM_SITE_MAX_DEPTH; return 0; }
  if (ps * 100 < P->min_ps) { c->cnt.min_ps_filter++; R->status = PM_SITE_MIN_PS; return 0; }
  if (avgmq < P->min_map_quality) { c->cnt.min_map_qual_filter++; R->status = PM_SITE_MIN_MAPQ; return 0; }

  const int ts = poly_ts(refBase), tv1 = poly_tv1(refBase), tv2 = poly_tv2(refBase);
  const double pts = P->poly_tstv / (P->poly_tstv + 1), ptv = (1 - pts) / 2, prior = c->prior;
  double varllk[7], noprior[7], varfreq[7];
  for (int k = 0; k < 7; k++) { varllk[k] = 0; noprior[k] = 0; varfreq[k] = 0; c->lk[k].evals = 0; }
  const int pa[7] = {0, refBase, refBase, refBase, ts, ts, tv1}, pb[7] = {0, ts, tv1, tv2, tv1, tv2, tv2};
  int maxidx; double vpp, qual;

  if (P->quick_call) {   /* main.cpp:354-437 */
    c->unrelated = 1;
    double v[7];
#pragma omp parallel sections
    {
#pragma omp section
      v[0] = log10(1 - prior) + mono_loglik(c);
#pragma omp section
      v[1] = log10(prior * pts) + poly_loglik(c, &c->lk[1], refBase, ts);
#pragma omp section
      v[2] = log10(prior * ptv) + poly_loglik(c, &c->lk[2], refBase, tv1);
#pragma omp section
      v[3] = log10(prior * ptv) + poly_loglik(c, &c->lk[3], refBase, tv2);
    }
    maxidx = var_posterior(c, v, 4, &vpp, &qual);
    if (vpp < 0.99) {
#pragma omp parallel sections
      {
#pragma omp section
        v[4] = log10(prior * 0.001) + poly_loglik(c, &c->lk[4], pa[4], pb[4]);
#pragma omp section
        v[5] = log10(prior * 0.001) + poly_loglik(c, &c->lk[5], pa[5], pb[5]);
#pragma omp section
        v[6] = log10(prior * 0.001) + poly_loglik(c, &c->lk[6], pa[6], pb[6]);
      }
      maxidx = var_posterior(c, v, 7, &vpp, &qual);
    }
    c->unrelated = 0;
    if (g_brent_err) return PM_EBRENT;
    if (vpp < P->posterior || maxidx == 0) { R->status = PM_SITE_QUICK_SKIP; return 0; }
    for (int k = 0; k < 7; k++) c->lk[k].evals = 0;
  }

  lkobj *o0 = &c->lk[0];
  /* the four configurations as the reference's `omp parallel sections` (main.cpp:439-495; a serial build runs them in
   * order); each has its own lkobj and, under OpenMP, the thread's own objective scratch */
#pragma omp parallel sections
  {
#pragma omp section
    {
      if (!c->denovo) {
        varllk[0] = log10(1 - prior) + mono_loglik(c);
      } else {
        /* FamilyLikelihoodSeq::MonomorphismLogLikelihood_denovo, FamilyLikelihoodSeq.cpp:68-72 */
        set_alleles(c, o0, refBase, refBase == 4 ? refBase - 1 : refBase + 1);
        o0->evals++;
        varllk[0] = log10(1 - prior) + all_fam_loglik(c, o0, 1.0);
      }
      noprior[0] = varllk[0] - log10(1 - prior); varfreq[0] = 1.0;
    }
#pragma omp section
    {
      varllk[1] = log10(prior * pts) + poly_loglik(c, &c->lk[1], refBase, ts);
      noprior[1] = varllk[1] - log10(prior * 2. / 3.); varfreq[1] = c->lk[1].min;
    }
#pragma omp section
    {
      varllk[2] = log10(prior * ptv) + poly_loglik(c, &c->lk[2], refBase, tv1);
      noprior[2] = varllk[2] - log10(prior * 1. / 6.); varfreq[2] = c->lk[2].min;
    }
#pragma omp section
    {
      varllk[3] = log10(prior * ptv) + poly_loglik(c, &c->lk[3], refBase, tv2);
      noprior[3] = varllk[3] - log10(prior * 1. / 6.); varfreq[3] = c->lk[3].min;
    }
  }
  maxidx = var_posterior(c, varllk, 4, &vpp, &qual);
  int ncfg = 4;
  if (vpp < 0.99) {   /* main.cpp:499-537 */
#pragma omp parallel for schedule(static, 1)
    for (int k = 4; k < 7; k++) {
      varllk[k] = log10(prior * 0.001) + poly_loglik(c, &c->lk[k], pa[k], pb[k]);
      noprior[k] = varllk[k] - log10(prior * 0.001);
      varfreq[k] = c->lk[k].min;
    }
    maxidx = var_posterior(c, varllk, 7, &vpp, &qual);
    ncfg = 7;
  }
  if (g_brent_err) return PM_EBRENT;
  R->status = PM_SITE_CALLED; R->n_cfg = ncfg; R->maxidx = maxidx; R->var_post_prob = vpp; R->poly_qual = qual;
  R->allele1 = c->lk[0].a1; R->allele2 = c->lk[0].a2;   /* set by CalcVarPosterior for every evaluated site */
  for (int k = 0; k < 7; k++) {
    R->varllk[k] = k < ncfg ? varllk[k] : 0.0; R->varfreq[k] = k < ncfg ? varfreq[k] : 0.0;
    R->evals[k] = k < ncfg ? (int32_t)c->lk[k].evals : 0;
  }

  /* main.cpp:539-594 */
  const int force = P->force_call, all = P->all_sites;
  if (vpp < P->posterior) { c->cnt.nocall++; if (!force && !all) return 0; }
  switch (maxidx) {
    case 0: c->cnt.homo_ref++; if (force || all) o0->min = 1.0; break;
    case 1: c->cnt.transitions++; set_alleles(c, o0, refBase, ts); o0->min = c->lk[1].min; break;
    case 2: c->cnt.transversions++; set_alleles(c, o0, refBase, tv1); o0->min = c->lk[2].min; break;
    case 3: c->cnt.transversions++; set_alleles(c, o0, refBase, tv2); o0->min = c->lk[3].min; break;
    case 4: c->cnt.tstvs1++; set_alleles(c, o0, ts, tv1); o0->min = c->lk[4].min; break;
    case 5: c->cnt.tstvs2++; set_alleles(c, o0, ts, tv2); o0->min = c->lk[5].min; break;
    default: c->cnt.tvs1tvs2++; set_alleles(c, o0, tv1, tv2); o0->min = c->lk[6].min; break;
  }
  if (maxidx == 0 && !c->denovo && !force && !all) return 0;
  double dlr = -1;
  if (maxidx == 0) {
    if (c->denovo) {
      double lk_mono = mono_loglik(c);
      o0->min = 1.0;
      dlr = noprior[0] - lk_mono;
      if (dlr <= log10(P->denovo_min_llr) && !all && !force) return 0;
    }
  } else if (c->denovo) {
    c->denovo = 0;
    long ev = o0->evals;
    double lk_poly = poly_loglik(c, o0, o0->a1, o0->a2);
    o0->evals = ev;
    dlr = noprior[maxidx] - lk_poly;
    c->denovo = 1;
    if (g_brent_err) return PM_EBRENT;
  }
  int denovo_mono = 0;
  if (maxidx == 0) {
    if (c->denovo) { denovo_mono = 1; calc_post_prob(c, 1.0); }
    else { o0->is_mono = 1; calc_post_prob(c, 1 - P->theta); }
  } else { o0->is_mono = 0; calc_post_prob(c, o0->min); }

  R->allele1 = o0->a1; R->allele2 = o0->a2; R->is_mono = c->denovo ? 0 : o0->is_mono;
  R->denovo_mono = denovo_mono; R->af = o0->min; R->denovo_lr = dlr;
  R->ab = (!c->isX && !c->isY && !c->isMT && !c->denovo) ? calc_ab(c, o0, o0->min) : 0.5;
  /* OutputVCF_denovo suppresses the record (header only) when denovoLR < minLLR (:1868) */
  R->emit = (c->denovo && dlr < P->denovo_min_llr) ? 2 : 1;
  R->call_row = 0;
  fill_calls(c, calls);
  return 0;
}
