/* feature_pool.h -- the local feature pool: a fixed-capacity open-addressing
 * hash map from BoW word id to the local feature seen under it (the last MAX_LOCAL_FRAMES
 * frames it was observed in, and its 3-D point), which a local-BA window consumes.
 *
 * Drop-in for include/local_feature_pool.h of the reference (header-only C there, with
 * non-static definitions, so a program can include it once).  The structs below have the
 * reference's layout field for field (LocalFeature :16-22, HashEntry :64-68,
 * LocalFeaturePool :82-86), so these functions also operate on a reference-allocated pool.
 * Semantics are the reference's, including the table layout: linear probing from
 * key % capacity (:93-131), deletion by the reference's backward-shift chain replacement
 * (:137-191), and the pruning walk of local_feature_pool_remove_old (:258-269), which
 * re-examines a slot after a deletion moved another entry into it.  Where the reference
 * exit()s (deleting a missing key :176-180, a broken invariant :279-336) these return an
 * error code instead.
 *
 * A flaw kept for parity: the refill rule (:143-159) moves an entry back into the vacated
 * slot only if its home slot is at or before the hole -- before the scan wraps past the
 * last slot -- so an entry whose own probe wrapped around the table end (home near
 * capacity - 1, stored just after a hole near slot 0) is never moved back.  When the hole
 * is then left empty that key becomes unreachable; its later deletion (pruning) fails,
 * which in the reference prints "Key not found" and exits.  The reference's own workload
 * (src/local_feature_matching.c, load <= 0.45) never builds such a cluster; random ids at
 * ~0.8 load, or ids crowded on homes around the wrap, do.  The layouts here are the reference's up to that point, and
 * mv_local_feature_pool_remove_old / _track_frame return MV_ERR_INVALID_ARG at it.
 *
 * Host code: the pool is a 3000-entry sequential structure (one frame's 200 inserts
 * depend on each other through the probe sequence), latency-bound on a CPU core; there is
 * no data-parallel work in it for the GPU.  mv_local_feature_pool_track_frame is the
 * per-frame step of src/local_feature_matching.c:151-164 (the reference's "MEASURE THIS"
 * block): insert each id or add the frame to the feature already there, then prune. */
#ifndef MV_FEATURE_POOL_H
#define MV_FEATURE_POOL_H

#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MV_MAX_LOCAL_FRAMES 8                /* local_feature_pool.h:11 */
#define MV_LOCAL_FEATURE_POOL_CAPACITY 3000  /* :14 */

typedef struct {
    int word_id; /* -1: empty */
    int frame_ptr;
    int num_frames;
    int frames[MV_MAX_LOCAL_FRAMES]; /* ring, oldest at frame_ptr */
    float coords_3D[3];
} mv_local_feature;

typedef struct {
    int key;
    mv_local_feature value;
    bool is_occupied;
} mv_lfp_entry;

typedef struct {
    mv_lfp_entry entries[MV_LOCAL_FEATURE_POOL_CAPACITY];
    int size;
    int capacity;
} mv_local_feature_pool;

/* init_local_feature / init_local_feature_with_id / update_local_feature /
 * remove_old_frame (:24-62): the per-feature frame ring */
void mv_local_feature_init(mv_local_feature *f);
void mv_local_feature_init_with_id(mv_local_feature *f, int word_id, int frame_num);
void mv_local_feature_update(mv_local_feature *f, int frame_num);
bool mv_local_feature_remove_old_frame(mv_local_feature *f, int oldest_keep_frame);

/* init_local_feature_pool (:97-103) */
void mv_local_feature_pool_init(mv_local_feature_pool *pool);
/* local_feature_pool_insert (:108-131): *feature = the entry's value (NULL when the pool is
 * full), *inserted = whether key was new.  Returns MV_OK, or MV_ERR_CAPACITY when full. */
int mv_local_feature_pool_insert(mv_local_feature_pool *pool, int key, const mv_local_feature *value,
                                 mv_local_feature **feature, bool *inserted);
/* local_feature_pool_delete (:170-191); MV_ERR_INVALID_ARG when key is absent (the
 * reference exits) */
int mv_local_feature_pool_delete(mv_local_feature_pool *pool, int key);
/* local_feature_pool_remove_old (:258-269): MV_OK, or MV_ERR_INVALID_ARG where a pruned
 * key is unreachable (the reference exits there; see above) */
int mv_local_feature_pool_remove_old(mv_local_feature_pool *pool, int current_frame_num);
/* local_feature_pool_valid_keys (:271-277): appends the occupied keys in slot order */
void mv_local_feature_pool_valid_keys(const mv_local_feature_pool *pool, int *num_keys, int *keys);
/* local_feature_pool_load_factor (:253-255) */
float mv_local_feature_pool_load_factor(const mv_local_feature_pool *pool);
/* local_feature_pool_check_invariant's checks (:279-336) without the printing: MV_OK, or
 * MV_ERR_INVALID_ARG on the first violation */
int mv_local_feature_pool_check_invariant(const mv_local_feature_pool *pool, int cur_frame);
/* one frame of src/local_feature_matching.c:153-164: for each of the n word ids in order,
 * insert a feature first seen at frame_num or add frame_num to the existing one, then
 * remove_old(frame_num).  Returns MV_OK, MV_ERR_CAPACITY if an insert found the pool
 * full (the reference would then dereference NULL), or remove_old's error. */
int mv_local_feature_pool_track_frame(mv_local_feature_pool *pool, int frame_num, int n, const int *word_ids);

#ifdef __cplusplus
}
#endif
#endif
