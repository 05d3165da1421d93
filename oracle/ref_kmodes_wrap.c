/* TEST INFRASTRUCTURE: System V wrappers around the reference asm (MS x64 ABI) built by
 * build_ref_asm.sh.  Signatures follow kmodes.pas:316 and kmodes.pas:455. */
#include <stdint.h>

extern int64_t __attribute__((ms_abi)) ref_GetMinMatchingDissim_Asm(const uint8_t *item, const uint8_t **list,
                                                                     uint64_t count, uint64_t *pbest);
extern void __attribute__((ms_abi)) ref_UpdateMinDistance_Asm(const uint8_t *item, const uint8_t **list,
                                                             const uint8_t *used, uint64_t *mindist, int count);

int64_t ref_get_min(const uint8_t *item, const uint8_t **list, uint64_t count, uint64_t *best) {
    return ref_GetMinMatchingDissim_Asm(item, list, count, best);
}

void ref_update_min_distance(const uint8_t *item, const uint8_t **list, const uint8_t *used, uint64_t *mindist,
                             int count) {
    ref_UpdateMinDistance_Asm(item, list, used, mindist, count);
}
