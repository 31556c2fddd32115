// oracle/ref/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never linked by the product).
//
// A driver of our own that links the *unmodified* reference objects (compiled in place from
// /root/reference/{core,src}, see oracle/ref/Makefile) and walks the per-site loop the way the
// reference CLI does (src/main.cpp:300-594).  The reference's main.cpp itself cannot be built in
// this image (it includes PedVCF.h -> libVcf -> tabix/bgzf/pcre which are absent), so this harness
// re-states its control flow against the reference's own classes:
//   Pedigree / PedigreeGLF / FamilyLikelihoodSeq / NucFamGenotypeLikelihood / FamilyLikelihoodES.
// It is pinned by reproducing the reference's committed goldens (example/test.out.vcf,
// test.denovo.out.vcf, test.out.vcfa) byte-for-byte outside the '##' header lines.
//
// Extra outputs (for kernel-level parity fixtures):
//   --dump_sites FILE : per processed site, a fixed binary record (see struct SiteDump below) with
//                       varllk[7], varfreq[7], per-config objective-evaluation counts, maxidx, ...
//   --dump_block FILE : the dense per-site input block as the reference's reader sees it
//                       (refBase, pos, then per person in VCF column order: 10 PL bytes, depth u32,
//                       mapQ u8), i.e. exactly what glfHandler::Get*(currentPos) return.
#include "FamilyLikelihoodSeq.h"
#include "NucFamGenotypeLikelihood.h"
#include "PedigreeGLF.h"
#include "Parameters.h"
#include "StringMap.h"
#include "CmdLinePar.h"
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <map>
#include <string>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

// FamilyLikelihoodSeq with an evaluation counter on the Brent objective (virtual f()).
class CountingFamLk : public FamilyLikelihoodSeq {
 public:
  long evals;
  CountingFamLk() : evals(0) {}
  virtual double f(double freq) { evals++; return FamilyLikelihoodSeq::f(freq); }
};

#pragma pack(push, 1)
struct SiteDump {
  int32_t pos;          // 1-based position
  int32_t refBase;      // 1..4
  int32_t status;       // 0 = evaluated, 1..4 = filtered (minDepth,maxDepth,minPS,minMapQ), 5 = bad refBase, 6 = skipped by --pos
  int32_t totalDepth;
  int32_t numSampWithData;
  double  avgMapQual;
  double  percSampWithData;
  int32_t n_cfg;        // 4 or 7
  int32_t maxidx;
  double  varPostProb;
  double  polyQual;
  double  varllk[7];
  double  varfreq[7];
  int32_t evals[7];     // objective evaluations per config (0 for mono)
  int32_t emitted;      // 1 if a VCF record was produced
  double  denovoLR;
};
#pragma pack(pop)

static StringArray g_glfNames;

static int LoadGlfIndex(const String& path, StringMap* map) {
  IFILE fh = ifopen(path.c_str(), "r");
  if (fh == NULL) error("%s open failed\n", path.c_str());
  String line; StringArray tok; int n = 0;
  while (!ifeof(fh)) {
    line.ReadLine(fh); tok.Clear(); tok.ReplaceTokens(line);
    if (tok.Length() < 2) continue;
    g_glfNames.Add(tok[1]);
    map->Add(tok[0], &g_glfNames[n]);
    n++;
  }
  ifclose(fh);
  return n;
}

static void LoadPositions(const String& file, std::map<String, int>& pos) {
  FILE* fh = fopen(file.c_str(), "r");
  if (fh == NULL) error("Open position file %s failed!\n", file.c_str());
  String buf; StringArray tok;
  while (!feof(fh)) {
    buf.ReadLine(fh); tok.ReplaceTokens(buf);
    if (tok.Length() == 0) continue;
    String key = tok[0] + ":" + tok[1];
    pos[key]++;
  }
  fclose(fh);
}

int main(int argc, char* argv[]) {
  double posterior = 0.5; int minTotalDepth = 0, maxTotalDepth = 0; double minPS = 0; int minMapQuality = 0;
  String pedFile, datFile, glfListFile, vcfOutFile = "", vcfInFile = "", positionfile, chrs2process;
  double theta = 0.001, theta_indel = 0.0001, tstv_ratio = 2.0, precision = 0.0001;
  int num_threads = 1; bool denovo = false; double denovo_mut_rate = 1.5e-08, denovo_tstv_ratio = 2.0, denovoLRmin = 0.01;
  bool gl_off = false, quick_call = false, force_call = false, out_all_sites = false, use_ext = false;
  String chrX_label("X"), chrY_label("Y"), MT_label("MT");
  String dumpSites, dumpBlock;

  ParameterList pl;
  BEGIN_LONG_PARAMETERS(lp)
    LONG_PARAMETER_GROUP("Alternative input file")
      LONG_STRINGPARAMETER("in_vcf", &vcfInFile)
    LONG_PARAMETER_GROUP("Scaled mutation rate")
      LONG_DOUBLEPARAMETER("theta", &theta)
      LONG_DOUBLEPARAMETER("indel_theta", &theta_indel)
    LONG_PARAMETER_GROUP("Prior of ts/tv ratio")
      LONG_DOUBLEPARAMETER("poly_tstv", &tstv_ratio)
    LONG_PARAMETER_GROUP("Non-autosome labels")
      LONG_STRINGPARAMETER("chrX", &chrX_label)
      LONG_STRINGPARAMETER("chrY", &chrY_label)
      LONG_STRINGPARAMETER("MT", &MT_label)
    LONG_PARAMETER_GROUP("de novo mutation")
      LONG_PARAMETER("denovo", &denovo)
      LONG_DOUBLEPARAMETER("rate_denovo", &denovo_mut_rate)
      LONG_DOUBLEPARAMETER("tstv_denovo", &denovo_tstv_ratio)
      LONG_DOUBLEPARAMETER("minLLR_denovo", &denovoLRmin)
    LONG_PARAMETER_GROUP("Optimization precision")
      LONG_DOUBLEPARAMETER("prec", &precision)
    LONG_PARAMETER_GROUP("Multiple threading")
      LONG_INTPARAMETER("nthreads", &num_threads)
    LONG_PARAMETER_GROUP("Chromosomes to process")
      LONG_STRINGPARAMETER("chr2process", &chrs2process)
    LONG_PARAMETER_GROUP("Filters")
      LONG_INTPARAMETER("minMapQuality", &minMapQuality)
      LONG_INTPARAMETER("minDepth", &minTotalDepth)
      LONG_INTPARAMETER("maxDepth", &maxTotalDepth)
      LONG_DOUBLEPARAMETER("minPercSampleWithData", &minPS)
    LONG_PARAMETER_GROUP("Output")
      LONG_STRINGPARAMETER("out_vcf", &vcfOutFile)
      LONG_STRINGPARAMETER("pos", &positionfile)
      LONG_PARAMETER("all_sites", &out_all_sites)
      LONG_PARAMETER("gl_off", &gl_off)
      LONG_PARAMETER("quick_call", &quick_call)
    LONG_PARAMETER_GROUP("Harness")
      LONG_PARAMETER("ext", &use_ext)
      LONG_STRINGPARAMETER("dump_sites", &dumpSites)
      LONG_STRINGPARAMETER("dump_block", &dumpBlock)
  END_LONG_PARAMETERS();
  pl.Add(new StringParameter('p', "pedfile", pedFile));
  pl.Add(new StringParameter('d', "datfile", datFile));
  pl.Add(new StringParameter('g', "glfIndexFile", glfListFile));
  pl.Add(new DoubleParameter('c', "posterior cutoff", posterior));
  pl.Add(new LongParameters("Additional Options", lp));
  pl.Read(argc, argv);
  pl.Status();

  if (vcfInFile.Length() > 0) error("the --in_vcf path is not buildable here (tabix/pcre absent)\n");
  if (pedFile.Length() == 0) error("pedFile not provided for input!\n");
  if (glfListFile.Length() == 0) error("glfListFile or input VCF file not provided for input!\n");
  if (vcfOutFile.Length() == 0) error("vcfOutFile not provided for output!\n");

  std::map<String, int> positionMap;
  if (positionfile.Length() > 0) { LoadPositions(positionfile, positionMap); force_call = true; quick_call = false; out_all_sites = false; }
  if (out_all_sites) quick_call = false;
#ifdef _OPENMP
  if (num_threads > 0) omp_set_num_threads(num_threads);
#endif
  std::string cmd;
  for (int a = 0; a < argc; a++) { cmd += argv[a]; cmd += " "; }

  CmdLinePar par;
  par.cmd = cmd; par.theta = theta; par.theta_indel = theta_indel;
  par.minTotalDepth = minTotalDepth; par.maxTotalDepth = maxTotalDepth; par.minMapQuality = minMapQuality;
  par.minPS = minPS; par.posterior = posterior; par.precision = precision;
  par.denovo_mut_rate = denovo_mut_rate; par.denovo_tstv_ratio = denovo_tstv_ratio; par.denovo = denovo;
  par.denovoLR = denovoLRmin; par.gl_off = gl_off; par.chrX_label = chrX_label; par.chrY_label = chrY_label;
  par.MT_label = MT_label; par.vcfInFile = vcfInFile; par.vcfOutFile = vcfOutFile;
  par.force_call = force_call; par.out_all_sites = out_all_sites;
  if (denovo && denovoLRmin < 0) error("denovo_min_LLR can only be greater than 0 !\n");

  const double p_ts = tstv_ratio / (tstv_ratio + 1);
  const double p_tv = (1 - p_ts) / 2;

  StringMap glfMap;
  LoadGlfIndex(glfListFile, &glfMap);
  Pedigree ped; PedigreeGLF pedGLF;
  IFILE datFH = ifopen(datFile, "r");
  IFILE pedFH = ifopen(pedFile, "r");
  FILE* vcfFH = fopen(vcfOutFile, "w");
  if (datFH == NULL) error("datFile open for input failed!\n");
  if (pedFH == NULL) error("pedFile open for input failed!\n");
  if (vcfFH == NULL) error("vcfOutFile can not be opened for output!\n");
  ped.Prepare(datFH);
  ped.Load(pedFH);
  if (use_ext) for (int f = 0; f < ped.familyCount; f++) ped.families[f]->generations = 3;
  ifclose(datFH); ifclose(pedFH);
  pedGLF.SetGLFMap(&glfMap);
  pedGLF.SetPedGLF(&ped);

  CountingFamLk lk[7];
  for (int r = 0; r < 7; r++) {
    lk[r].SetCmdLinePar(&par);
    if (denovo) lk[r].SetDenovoMutationModel();
    lk[r].SetTheta(theta);
    lk[r].SetTheta_indel(theta_indel);
    lk[r].SetGLF(&pedGLF);
    lk[r].InitFamilyLikelihoodES();
    if (quick_call) lk[r].BackupFounderCount();
  }

  FILE* dsFH = dumpSites.Length() ? fopen(dumpSites, "wb") : NULL;
  FILE* dbFH = dumpBlock.Length() ? fopen(dumpBlock, "wb") : NULL;

  std::map<String, int> chrSel;
  { StringArray chrs; chrs.AddTokens(chrs2process, ','); for (int i = 0; i < chrs.Length(); i++) chrSel[chrs[i]]++; }
  int chrSelCount = chrSel.size();

  time_t t0; time(&t0);
  printf("Analysis started on %s\n", ctime(&t0));
  int chrDone = 0, out_cnt = 0;
  NucFamGenotypeLikelihood& m0 = lk[0];

  while (pedGLF.Move2NextSection()) {
    if (chrSel.size() > 0 && chrDone >= chrSelCount) break;
    String label = pedGLF.GetNonNULLglf()->label;
    if (chrSel.size() > 0 && chrSel[label] < 1) { while (pedGLF.Move2NextBaseEntry()) {} continue; }
    bool isX = label == par.chrX_label, isY = !isX && label == par.chrY_label, isMT = !isX && !isY && label == par.MT_label;
    for (int r = 0; r < 7; r++) lk[r].SetNonAutosomeFlags(isX, isY, isMT);

    int homoRef = 0, nTs = 0, nTv = 0, c_tstv1 = 0, c_tstv2 = 0, c_tv1tv2 = 0, nocall = 0, entries = 0;
    int baseCounts[5] = {0, 0, 0, 0, 0};
    unsigned fMinDepth = 0, fMaxDepth = 0, fMinMQ = 0, fMinPS = 0;
    double polyPrior = lk[0].GetPolyPrior();
    double polyPrior_unr = lk[0].GetPolyPrior_unr();
    chrDone++;

    while (pedGLF.Move2NextBaseEntry()) {
      for (int r = 0; r < 7; r++) lk[r].FillPenetrance();
      if (entries == 0) entries = pedGLF.GetNonNULLglf()->maxPosition;

      SiteDump sd; memset(&sd, 0, sizeof(sd));
      sd.pos = pedGLF.currentPos + 1;
      sd.refBase = pedGLF.GetRefBase();
      sd.maxidx = -2;

      if (positionfile.Length() > 0) {
        String key = label + ":" + (pedGLF.currentPos + 1);
        if (positionMap.count(key) == 0) { sd.status = 6; if (dsFH) fwrite(&sd, sizeof(sd), 1, dsFH); continue; }
      }
      int refBase = pedGLF.GetRefBase();
      if (dbFH) {
        int32_t hdr[2] = {pedGLF.currentPos + 1, refBase};
        fwrite(hdr, sizeof(hdr), 1, dbFH);
        for (int i = 0; i < ped.familyCount; i++)
          for (int j = 0; j < ped.families[i]->count; j++) {
            glfHandler& g = pedGLF.glf[i][j];
            unsigned char pl10[10]; uint32_t dp = 0; unsigned char mq = 0;
            if (g.handle == NULL) { memset(pl10, 0, 10); }
            else {
              memcpy(pl10, g.GetLogLikelihoods(pedGLF.currentPos), 10);
              dp = g.GetDepth(pedGLF.currentPos); mq = g.GetMapQuality(pedGLF.currentPos);
            }
            fwrite(pl10, 10, 1, dbFH); fwrite(&dp, 4, 1, dbFH); fwrite(&mq, 1, 1, dbFH);
          }
      }
      if (refBase != 1 && refBase != 2 && refBase != 3 && refBase != 4) { sd.status = 5; if (dsFH) fwrite(&sd, sizeof(sd), 1, dsFH); continue; }
      baseCounts[refBase]++;

      m0.CalcReadStats();
      sd.totalDepth = m0.totalDepth; sd.numSampWithData = m0.numSampWithData;
      sd.avgMapQual = m0.avgMapQual; sd.percSampWithData = m0.percSampWithData;
      int filt = 0;
      if (m0.totalDepth < minTotalDepth) { fMinDepth++; filt = 1; }
      else if (maxTotalDepth > 0 && m0.totalDepth > maxTotalDepth) { fMaxDepth++; filt = 2; }
      else if (m0.percSampWithData * 100 < minPS) { fMinPS++; filt = 3; }
      else if (m0.avgMapQual < minMapQuality) { fMinMQ++; filt = 4; }
      if (filt) { sd.status = filt; if (dsFH) fwrite(&sd, sizeof(sd), 1, dsFH); continue; }

      const int ts = Poly::ts(refBase), tv1 = Poly::tvs1(refBase), tv2 = Poly::tvs2(refBase);
      for (int r = 0; r < 7; r++) lk[r].evals = 0;
      int maxidx = 0;

      if (quick_call) {
        for (int r = 0; r < 7; r++) lk[r].MakeUnrelated();
        // main.cpp:361-393 / 401-426: `omp parallel sections` over the configurations, as the reference
#pragma omp parallel sections
        {
#pragma omp section
          m0.varllk[0] = log10(1 - polyPrior_unr) + lk[0].MonomorphismLogLikelihood(refBase);
#pragma omp section
          m0.varllk[1] = log10(polyPrior_unr * p_ts) + lk[1].PolymorphismLogLikelihood(refBase, ts);
#pragma omp section
          m0.varllk[2] = log10(polyPrior_unr * p_tv) + lk[2].PolymorphismLogLikelihood(refBase, tv1);
#pragma omp section
          m0.varllk[3] = log10(polyPrior_unr * p_tv) + lk[3].PolymorphismLogLikelihood(refBase, tv2);
        }
        maxidx = m0.CalcVarPosterior(4);
        if (m0.varPostProb < 0.99) {
#pragma omp parallel sections
          {
#pragma omp section
            m0.varllk[4] = log10(polyPrior_unr * 0.001) + lk[4].PolymorphismLogLikelihood(ts, tv1);
#pragma omp section
            m0.varllk[5] = log10(polyPrior_unr * 0.001) + lk[5].PolymorphismLogLikelihood(ts, tv2);
#pragma omp section
            m0.varllk[6] = log10(polyPrior_unr * 0.001) + lk[6].PolymorphismLogLikelihood(tv1, tv2);
          }
          maxidx = m0.CalcVarPosterior(7);
        }
        if (m0.varPostProb < posterior || maxidx == 0) { sd.status = 7; if (dsFH) fwrite(&sd, sizeof(sd), 1, dsFH); continue; }
        for (int r = 0; r < 7; r++) lk[r].RestoreFounderCount();
        for (int r = 0; r < 7; r++) lk[r].evals = 0;
      }

      // Most likely configurations: monomorphic + the three ref/alt pairs, as the reference's 4 `omp parallel
      // sections` (main.cpp:439-495; the family loops inside them are inactive nested regions)
#pragma omp parallel sections
      {
#pragma omp section
        {
          if (!par.denovo) {
            double l = log10(1 - polyPrior) + lk[0].MonomorphismLogLikelihood(refBase);
            m0.varllk[0] = l; m0.varllk_noprior[0] = l - log10(1 - polyPrior); m0.varfreq[0] = 1.0;
          } else {
            double l = log10(1 - polyPrior) + lk[0].MonomorphismLogLikelihood_denovo(refBase, refBase == 4 ? refBase - 1 : refBase + 1);
            m0.varllk[0] = l; m0.varllk_noprior[0] = l - log10(1 - polyPrior); m0.varfreq[0] = 1.0;
          }
        }
#pragma omp section
        {
          double l = log10(polyPrior * p_ts) + lk[1].PolymorphismLogLikelihood(refBase, ts);
          m0.varllk[1] = l; m0.varllk_noprior[1] = l - log10(polyPrior * 2. / 3.); m0.varfreq[1] = lk[1].GetMinimizer();
        }
#pragma omp section
        {
          double l = log10(polyPrior * p_tv) + lk[2].PolymorphismLogLikelihood(refBase, tv1);
          m0.varllk[2] = l; m0.varllk_noprior[2] = l - log10(polyPrior * 1. / 6.); m0.varfreq[2] = lk[2].GetMinimizer();
        }
#pragma omp section
        {
          double l = log10(polyPrior * p_tv) + lk[3].PolymorphismLogLikelihood(refBase, tv2);
          m0.varllk[3] = l; m0.varllk_noprior[3] = l - log10(polyPrior * 1. / 6.); m0.varfreq[3] = lk[3].GetMinimizer();
        }
      }
      maxidx = m0.CalcVarPosterior(4);
      sd.n_cfg = 4;
      if (m0.varPostProb < 0.99) {
        const int pa[3] = {ts, ts, tv1}, pb[3] = {tv1, tv2, tv2};
#pragma omp parallel for schedule(static, 1)   // main.cpp:501-535: three sections
        for (int k = 0; k < 3; k++) {
          double l = log10(polyPrior * 0.001) + lk[4 + k].PolymorphismLogLikelihood(pa[k], pb[k]);
          m0.varllk[4 + k] = l; m0.varllk_noprior[4 + k] = l - log10(polyPrior * 0.001);
          m0.varfreq[4 + k] = lk[4 + k].GetMinimizer();
        }
        maxidx = m0.CalcVarPosterior(7);
        sd.n_cfg = 7;
      }
      sd.maxidx = maxidx; sd.varPostProb = m0.varPostProb; sd.polyQual = m0.polyQual;
      for (int k = 0; k < 7; k++) { sd.varllk[k] = m0.varllk[k]; sd.varfreq[k] = m0.varfreq[k]; sd.evals[k] = (int)lk[k].evals; }
      // lk[0].evals counts objective calls of the mono/de-novo-mono evaluation (0 or 1).

      bool skip = false;
      if (m0.varPostProb < posterior) { nocall++; if (!force_call && !out_all_sites) skip = true; }
      if (!skip) {
        switch (maxidx) {
          case 0: homoRef++; if (force_call || out_all_sites) m0.min = 1.0; break;
          case 1: nTs++; m0.SetAlleles(refBase, ts); m0.min = lk[1].min; break;
          case 2: nTv++; m0.SetAlleles(refBase, tv1); m0.min = lk[2].min; break;
          case 3: nTv++; m0.SetAlleles(refBase, tv2); m0.min = lk[3].min; break;
          case 4: c_tstv1++; m0.SetAlleles(ts, tv1); m0.min = lk[4].min; break;
          case 5: c_tstv2++; m0.SetAlleles(ts, tv2); m0.min = lk[5].min; break;
          case 6: c_tv1tv2++; m0.SetAlleles(tv1, tv2); m0.min = lk[6].min; break;
          case -1: nocall++; break;
          default: error("Invalid maxidx!\n");
        }
        if (maxidx == -1 || (maxidx == 0 && !par.denovo && !force_call && !out_all_sites)) skip = true;
      }
      if (!skip) {
        if (maxidx == 0) {
          if (par.denovo) {
            double lk_mono = lk[0].MonomorphismLogLikelihood(refBase);
            m0.min = 1.0;
            m0.denovoLR = m0.varllk_noprior[0] - lk_mono;
            if (m0.denovoLR <= log10(par.denovoLR) && !out_all_sites && !force_call) skip = true;
          }
        } else if (par.denovo) {
          par.denovo = false;
          double lk_poly = lk[0].PolymorphismLogLikelihood(m0.allele1, m0.allele2);
          m0.denovoLR = m0.varllk_noprior[maxidx] - lk_poly;
          par.denovo = true;
        }
      }
      if (!skip) {
        if (maxidx == 0) {
          if (par.denovo) { m0.denovo_mono = true; lk[0].CalcPostProb(1.0); }
          else { m0.isMono = true; lk[0].CalcPostProb(1 - theta); }
        } else { m0.isMono = false; lk[0].CalcPostProb(m0.min); }
        denovo ? m0.OutputVCF_denovo(vcfFH) : m0.OutputVCF(vcfFH);
        m0.denovo_mono = false;
        sd.emitted = 1; sd.denovoLR = m0.denovoLR;
        out_cnt++;
      }
      if (dsFH) fwrite(&sd, sizeof(sd), 1, dsFH);
      if (!skip && force_call && out_cnt >= (int)positionMap.size()) { if (dsFH) fclose(dsFH); if (dbFH) fclose(dbFH); return 0; }
    }

    int total = 0;
    for (int i = 0; i < 5; i++) total += baseCounts[i];
    printf("Summary of reference -- %s\n", label.c_str());
    printf("Total Entry Count: %9d\n", entries);
    printf("Total Base Cout: %9d\n", total);
    printf("Non-Polymorphic Count: %9d\n", homoRef);
    printf("Transition Count: %9d\n", nTs);
    printf("Transversion Count: %9d\n", nTv);
    printf("Other Polymorphism Count: %9d\n", c_tstv1 + c_tstv2 + c_tv1tv2);
    printf("Filter counts:\n");
    printf("\tminMapQual %u\n", fMinMQ);
    printf("\tminTotalDepth %u\n", fMinDepth);
    printf("\tmaxTotalDepth %u\n", fMaxDepth);
    printf("Hard to call: %9d\n", nocall);
    printf("Skipped bases: %u\n", entries - homoRef - nTs - nTv - (c_tstv1 + c_tstv2 + c_tv1tv2));
    time_t t1; time(&t1);
    printf("Analysis ended on %s\n", ctime(&t1));
    printf("Running time is %u seconds\n\n", (unsigned int)(t1 - t0));
    fflush(vcfFH);
  }
  fclose(vcfFH);
  if (dsFH) fclose(dsFH);
  if (dbFH) fclose(dbFH);
  return 0;
}
