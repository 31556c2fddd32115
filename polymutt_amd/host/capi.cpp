// capi.cpp -- C ABI of the host helpers (include/polymutt_host.h).
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include "../../include/polymutt_host.h"
#include "../csrc/synth_core.h"
#include "driver.h"
#include "engine_eval.h"
#include "glf.h"
#include "pedigree.h"
#include "synth.h"

extern "C" void pm_set_last_error(const char* msg);   // defined with the engine (thread-local)

struct pmh_pedigree { pmhost::Pedigree ped; };
struct pmh_glf_reader { pmhost::SiteSource src; bool started = false; bool in_section = false; };

extern "C" {

pmh_pedigree* pmh_pedigree_load(const char* dat, const char* ped) {
  try {
    auto* p = new pmh_pedigree;
    p->ped.load(dat, ped);
    return p;
  } catch (const std::exception& e) {
    pm_set_last_error(e.what());
    return nullptr;
  }
}

int pmh_pedigree_view(const pmh_pedigree* p, pm_pedigree* out) {
  if (!p || !out) { pm_set_last_error("pmh_pedigree_view: null argument"); return PM_EINVAL; }
  *out = p->ped.view();
  return PM_OK;
}

const char* pmh_pedigree_pid(const pmh_pedigree* p, int32_t person) {
  if (!p || person < 0 || person >= (int32_t)p->ped.column_pid.size()) return nullptr;
  return p->ped.column_pid[person].c_str();
}

const char* pmh_pedigree_famid(const pmh_pedigree* p, int32_t f) {
  if (!p || f < 0 || f >= (int32_t)p->ped.families.size()) return nullptr;
  return p->ped.families[f].famid.c_str();
}

int32_t pmh_pedigree_is_nuclear(const pmh_pedigree* p, int32_t f) {
  if (!p || f < 0 || f >= (int32_t)p->ped.families.size()) return -1;
  return p->ped.families[f].isNuclear() ? 1 : 0;
}

void pmh_pedigree_free(pmh_pedigree* p) { delete p; }

pmh_glf_reader* pmh_glf_open(const pmh_pedigree* p, const char* index) {
  try {
    auto* r = new pmh_glf_reader;
    r->src.open(p->ped, index);
    return r;
  } catch (const std::exception& e) {
    pm_set_last_error(e.what());
    return nullptr;
  }
}

int pmh_glf_next_section(pmh_glf_reader* r, char* label, int32_t cap, int32_t* max_position) {
  try {
    if (r->in_section) { int32_t pos; uint8_t ref; while (r->src.nextBaseEntry()) {} (void)pos; (void)ref; }
    if (!r->src.nextSection()) { r->in_section = false; return 0; }
    r->in_section = true;
    if (label && cap > 0) { strncpy(label, r->src.label().c_str(), cap - 1); label[cap - 1] = 0; }
    if (max_position) *max_position = r->src.maxPosition();
    return 1;
  } catch (const std::exception& e) {
    pm_set_last_error(e.what());
    return PM_EINVAL;
  }
}

int pmh_glf_read_sites(pmh_glf_reader* r, int32_t max_sites, int32_t* pos, uint8_t* ref, uint8_t* pl, uint32_t* dm) {
  if (!r->in_section) return 0;
  const int np = r->src.nPerson();
  int n = 0;
  while (n < max_sites && r->src.nextBaseEntry()) {
    pos[n] = r->src.currentPos + 1;
    ref[n] = (uint8_t)r->src.refBase;
    r->src.fill(pl + (size_t)n * np * 10, dm + (size_t)n * np);
    n++;
  }
  if (n < max_sites) r->in_section = false;
  return n;
}

void pmh_glf_close(pmh_glf_reader* r) { delete r; }

int pmh_run_polymutt(int argc, char** argv, int32_t rank, int32_t world, int32_t device, pmh_allgather_fn allgather, void* ctx) {
  pmhost::ShardComm comm;
  comm.rank = rank;
  comm.world = world;
  if (world > 1 || (world == 1 && allgather)) {   // (world 1 + allgather: the sharded protocol over one rank)
    if (!allgather || rank < 0 || rank >= world) { fprintf(stderr, "pmh_run_polymutt: invalid shard arguments\n"); return 1; }
    comm.allgather = [=](const int64_t* send, int n, int64_t* recv) {
      if (allgather(ctx, send, n, recv) != 0) throw pmhost::FatalError("shard exchange (allgather) failed\n");
    };
  }
  return pmhost::polymutt_main(argc, argv, &comm, [&](const pm_pedigree& v, const pm_params& par, const pmhost::Options& opt) {
    // (several engines only where batches are pipelined: one process, GLF or block input, no --pos; a shard, --pos or
    // --in_vcf run uses one -- run_polymutt_vcf evaluates on the first engine only)
    const int engines = (world > 1 || allgather || opt.force_call || !opt.vcfInFile.empty() || getenv("PM_SERIAL")) ? 1 : opt.engines;
    return std::unique_ptr<pmhost::SiteEvaluator>(
        new pmhost::EngineEvaluator(v, par, device >= 0 ? device : opt.device, opt.batch, engines));
  });
}

int pmh_synth_write_dataset(const char* dir, const char* shape, int32_t nfam, int32_t nsites, uint64_t seed) {
  std::string err;
  if (pmhost::synth_write_dataset(dir, shape, nfam, nsites, seed, err) != 0) { pm_set_last_error(err.c_str()); return PM_EINVAL; }
  return PM_OK;
}

int pmh_synth_block(const pm_pedigree* ped, int32_t n, uint64_t seed, uint64_t off, uint8_t* pl, uint32_t* dm, uint8_t* ref) {
  static pm_synth_tables T;
  static bool built = false;
  if (!built) { pm_synth_build_tables(&T); built = true; }
  const int np = ped->n_person;
  std::vector<int32_t> fa(np), mo(np);
  std::vector<uint8_t> hap(np);
  for (int f = 0; f < ped->n_fam; f++)
    for (int j = ped->fam_start[f]; j < ped->fam_start[f + 1]; j++) {
      fa[j] = ped->father[j] < 0 ? -1 : ped->father[j] - ped->fam_start[f];
      mo[j] = ped->mother[j] < 0 ? -1 : ped->mother[j] - ped->fam_start[f];
    }
  for (int i = 0; i < n; i++) {
    int r; double af;
    pm_syn_site(seed, off + i, &r, &af);
    ref[i] = (uint8_t)r;
    for (int f = 0; f < ped->n_fam; f++) {
      int s = ped->fam_start[f], cnt = ped->fam_start[f + 1] - s;
      pm_syn_family(&T, seed, off + i, r, af, cnt, fa.data() + s, mo.data() + s, (uint64_t)s, pl + ((size_t)i * np + s) * 10, 10, 1,
                    dm + (size_t)i * np + s, hap.data());
    }
  }
  return PM_OK;
}

}  // extern "C"
