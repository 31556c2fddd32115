// vcf.cpp -- see vcf.h.
#include "vcf.h"
#include <ctime>
#include "vcf_fmt.h"

namespace pmhost {

static const char kBases[5] = {'0', 'A', 'C', 'G', 'T'};
static const char* kGeno10[10] = {"A/A", "A/C", "A/G", "A/T", "C/C", "C/G", "C/T", "G/G", "G/T", "T/T"};

static int GI(int b1, int b2) {
  return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2);
}

bool VcfWriter::singleNuclear() const { return ped->families.size() == 1 && ped->families[0].isNuclear(); }

void VcfWriter::header() {
  time_t t; time(&t);
  fprintf(fh, "##fileformat=VCFv4.0\n");
  fprintf(fh, "##fileDate=%s", ctime(&t));
  fprintf(fh, "##command=%s\n", cmd.c_str());
  fprintf(fh, "##minMapQuality=%f\n", minMapQuality);
  fprintf(fh, "##minTotalDepth=%d\n", minTotalDepth);
  fprintf(fh, "##maxTodalDepth=%d\n", maxTotalDepth);
  fprintf(fh, "##posterior=%.3f\n", posterior);
  fprintf(fh, "##INFO=<ID=NS,Number=1,Type=Integer,Description=\"Number of Samples With Data\">\n");
  fprintf(fh, "##INFO=<ID=PS,Number=1,Type=Integer,Description=\"Percentage of Samples With Data\">\n");
  fprintf(fh, "##INFO=<ID=DP,Number=1,Type=Integer,Description=\"Total Read Depth\">\n");
  fprintf(fh, "##INFO=<ID=MQ,Number=1,Type=Float,Description=\"Average Map Quality\">\n");
  if (!singleNuclear()) fprintf(fh, "##INFO=<ID=AF,Number=.,Type=Float,Description=\"Reference Allele Frequency\">\n");
  if (denovo) fprintf(fh, "##INFO=<ID=DQ,Number=1,Type=Float,Description=\"De Novo Mutation Quality\">\n");
  fprintf(fh, "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n");
  fprintf(fh, "##FORMAT=<ID=GQ,Number=1,Type=Integer,Description=\"Genotype Quality\">\n");
  fprintf(fh, "##FORMAT=<ID=DP,Number=1,Type=Integer,Description=\"Read Depth\">\n");
  if (!denovo) fprintf(fh, "##FORMAT=<ID=DS,Number=1,Type=Float,Description=\"Dosage: Defined As the Expected Alternative Allele Count\">\n");
  if (!gl_off) fprintf(fh, "##FORMAT=<ID=PL,Number=10,Type=Integer,Description=\"Phred-scaled Genotype Likelhood\">\n");
  if (!denovo && force_call) fprintf(fh, "##FORMAT=<ID=BA,String,Description=\"Best Alterantive Allele\">\n");
  fprintf(fh, "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT");
  for (auto& pid : ped->column_pid) fprintf(fh, "\t%s", pid.c_str());
  fprintf(fh, "\n");
  if (denovo) fflush(fh);
  header_written = true;
}

void VcfWriter::output(const std::string& label, int pos1, int refBase, const pm_site_result& r, const pm_geno_call* calls,
                       const uint8_t* pl, const uint32_t* dm) {
  if (!header_written) header();
  if (r.emit != 1) return;   // OutputVCF_denovo returns before the record when denovoLR < minLLR (:1868)
  line_.clear();
  format(line_, label, pos1, refBase, r, calls, pl, dm);
  fwrite(line_.data(), 1, line_.size(), fh);
  fflush(fh);
}

void VcfWriter::format(std::string& L, const std::string& label, int pos1, int refBase, const pm_site_result& r,
                       const pm_geno_call* calls, const uint8_t* pl, const uint32_t* dm) const {
  const int n = (int)ped->column_pid.size();
  const bool refIsA1 = refBase == r.allele1;
  char info[512], head[1024];
  std::string alt;
  auto label_of = [&](const pm_geno_call& c) -> const char* {
    switch (c.label) {
      case PM_LBL_DOT: return ".";
      case PM_LBL_GENO10: return kGeno10[c.best];
      case PM_LBL_ALLELES: {
        int idx = c.best == 0 ? GI(r.allele1, r.allele1) : c.best == 1 ? GI(r.allele1, r.allele2) : GI(r.allele2, r.allele2);
        return kGeno10[idx];
      }
      default: {   // GetBestGenoLabel_vcfv4, :1590-1608
        static const char* dip[5] = {"0/0", "0/1", "1/1", "1/2", "2/2"};
        static const char* hap[5] = {"0", "ERROR", "1", "ERROR2", "2"};
        int li = c.best == 0 ? (refIsA1 ? 0 : 2) : c.best == 1 ? (refIsA1 ? 1 : 3) : (refIsA1 ? 2 : 4);
        return c.label == PM_LBL_VCF_HAPLOID ? hap[li] : dip[li];
      }
    }
  };
  if (!denovo) {
    const bool nonAuto = chrom != PM_CHR_AUTO;
    if (singleNuclear())
      snprintf(info, sizeof(info), "NS=%d;PS=%.1f;DP=%d;MQ=%.1f", r.num_samp_with_data, r.perc_samp_with_data * 100, r.total_depth, r.avg_map_qual);
    else if (nonAuto)
      snprintf(info, sizeof(info), "NS=%d;PS=%.1f;DP=%d;MQ=%.1f;AF=%.4f", r.num_samp_with_data, r.perc_samp_with_data * 100, r.total_depth, r.avg_map_qual, r.af);
    else
      snprintf(info, sizeof(info), "NS=%d;PS=%.1f;DP=%d;MQ=%.1f;AF=%.4f;AB=%.3f", r.num_samp_with_data, r.perc_samp_with_data * 100, r.total_depth,
               r.avg_map_qual, r.af, r.ab);
    std::string INFO = info;
    if (r.is_mono) { INFO += ";BA="; INFO += kBases[r.allele2]; }
    if (refIsA1) alt = std::string(1, kBases[r.is_mono ? r.allele1 : r.allele2]);
    else alt = std::string(1, kBases[r.allele1]) + "," + kBases[r.allele2];
    L += label;   // (the label and INFO appended whole: no length limit)
    snprintf(head, sizeof(head), "\t%d\t%s\t%c\t%s\t%d\t%s\t", pos1, ".", kBases[refBase], alt.c_str(), int(r.poly_qual + 0.5), ".");
    L += head;
    L += INFO;
    L += gl_off ? "\tGT:GQ:DP:DS" : "\tGT:GQ:DP:DS:PL";
    const int g11 = GI(r.allele1, r.allele1), g12 = GI(r.allele1, r.allele2), g22 = GI(r.allele2, r.allele2);
    // "\t%s:%d:%d:%.2f[:%u,%u,%u]" per person, formatted without stdio into reserved room (<= 96 chars a person)
    const size_t at = L.size();
    L.resize(at + (size_t)n * 96 + 2);
    char* o = &L[at];
    for (int p = 0; p < n; p++) {
      const pm_geno_call& c = calls[p];
      *o++ = '\t';
      put_str(o, label_of(c));
      *o++ = ':';
      put_int(o, (int)c.gq);
      *o++ = ':';
      put_uint(o, dm[p] & 0xFFFFFF);
      *o++ = ':';
      put_fixed2(o, c.dosage);
      if (!gl_off) {
        *o++ = ':'; put_uint(o, pl[p * 10 + g11]);
        *o++ = ','; put_uint(o, pl[p * 10 + g12]);
        *o++ = ','; put_uint(o, pl[p * 10 + g22]);
      }
    }
    *o++ = '\n';
    L.resize(o - L.data());
  } else {
    const int a2 = r.denovo_mono ? r.allele1 : r.allele2;
    if (singleNuclear())
      snprintf(info, sizeof(info), "NS=%d;PS=%.1f;DP=%d;MQ=%.1f;DQ=%.3f", r.num_samp_with_data, r.perc_samp_with_data * 100, r.total_depth,
               r.avg_map_qual, r.denovo_lr);
    else
      snprintf(info, sizeof(info), "NS=%d;PS=%.1f;DP=%d;MQ=%.1f;AF=%.4f;DQ=%.3f", r.num_samp_with_data, r.perc_samp_with_data * 100, r.total_depth,
               r.avg_map_qual, r.af, r.denovo_lr);
    if (refIsA1) alt = std::string(1, kBases[a2]);
    else alt = std::string(1, kBases[r.allele1]) + "," + kBases[a2];
    L += label;
    snprintf(head, sizeof(head), "\t%d\t%s\t%c\t%s\t%d\t%s\t%s\t%s", pos1, ".", kBases[refBase], alt.c_str(), int(r.poly_qual + 0.5), ".",
             info, gl_off ? "GT:GQ:DP" : "GT:GQ:DP:PL");
    L += head;
    const size_t at = L.size();
    L.resize(at + (size_t)n * 96 + 2);
    char* o = &L[at];
    for (int p = 0; p < n; p++) {
      const pm_geno_call& c = calls[p];
      *o++ = '\t';
      put_str(o, label_of(c));
      *o++ = ':';
      put_int(o, (int)c.gq);
      *o++ = ':';
      put_uint(o, dm[p] & 0xFFFFFF);
      if (!gl_off) {
        *o++ = ':';
        for (int g = 0; g < 9; g++) { put_uint(o, pl[p * 10 + g]); *o++ = ','; }
        put_uint(o, pl[p * 10 + 9]);
      }
    }
    *o++ = '\n';
    L.resize(o - L.data());
  }
}

}  // namespace pmhost
