/* apps/word2vec/word2vec.h under its reference name: the local variant of w2v_local.cpp (atoi
 * keys, each minibatch its own vocabulary and unigram table, word2vec.h:281-629) — see
 * word2vec_app.h. */
#ifndef SWIFTMPI_WORD2VEC_LOCAL_H_
#define SWIFTMPI_WORD2VEC_LOCAL_H_
#include "swiftmpi/apps/word2vec/word2vec_app.h"
template <typename MiniBatchT> using Word2Vec = swift_snails::Word2VecT<MiniBatchT, true>;
#endif
