// mh_fastq.h -- staged FASTQ text (mh_fastq.cpp) handed to the read loader.
#pragma once
#include <string>

#include "mh_gunzip.h"

struct mh_fastq;

namespace mh {
// move the held text out of a staged FASTQ (the handle keeps an empty text)
TextBuf take_fastq_text(mh_fastq *fq);
// the held text of a staged FASTQ
const TextBuf &fastq_text(const mh_fastq *fq);
}  // namespace mh
