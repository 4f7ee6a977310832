/* Host-side decoding library (libliteasr_decode.so), SURVEY §8 f3.
 *
 * lasr_ctc_prefix_beam_search replaces the pure-Python loop of
 * liteasr/models/u2.py:218-263 (`U2._ctc_prefix_beam_search`, with `log_add`
 * u2.py:367-375).  Its input is what the device kernel lasr_logsoftmax_topk
 * (liteasr_hip.h) leaves per frame: the k = beam largest CTC log-probs, descending, and
 * their token ids, [T, k] row-major.  Output: up to `beam` hypotheses, best first; their
 * tokens concatenated into out_tok (capacity cap_tok), lengths in out_len[beam], scores
 * log_add(pb, pnb) in out_score[beam].  Returns the number of hypotheses (>= 1), or a
 * negative code with lasr_decode_last_error() set.  Pure host code, reentrant. */
#ifndef LITEASR_DECODE_H
#define LITEASR_DECODE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int lasr_ctc_prefix_beam_search(const float* topk_val, const int32_t* topk_idx, int T, int k,
                                int blank, int beam, int32_t* out_tok, int64_t cap_tok,
                                int32_t* out_len, double* out_score);
const char* lasr_decode_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LITEASR_DECODE_H */
