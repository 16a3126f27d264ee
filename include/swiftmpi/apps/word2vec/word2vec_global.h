/* apps/word2vec/word2vec_global.h under its reference name: the global-vocabulary word2vec
 * (BKDR keys, one unigram table) of w2v.cpp — see word2vec_app.h. */
#ifndef SWIFTMPI_WORD2VEC_GLOBAL_H_
#define SWIFTMPI_WORD2VEC_GLOBAL_H_
#include "swiftmpi/apps/word2vec/word2vec_app.h"
/* the reference's minibatch worker (gather / pull / learn / push): the library's device loop */
class MiniBatch {};
template <typename MiniBatchT> using Word2Vec = swift_snails::Word2VecT<MiniBatchT, false>;
#endif
