/* Sequential restatement of the GPU BGZF block encoder -- TEST INFRASTRUCTURE ONLY (bgzf_ref.c). */
#ifndef BGZF_REF_H
#define BGZF_REF_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int bgzf_ref_block(const uint8_t *in, int n, uint8_t *out);
void bgzf_huffman_lengths(const uint32_t *freq, int n, int limit, uint8_t *len);
void bgzf_canonical_codes(const uint8_t *len, int n, uint16_t *code);
int bgzf_rle_lengths(const uint8_t *lens, int n, uint8_t *sym, uint8_t *ext);
#ifdef __cplusplus
}
#endif
#endif
