/* feature_pool.c -- the local feature pool (include/feature_pool.h), host code.
 *
 * Restates include/local_feature_pool.h of the reference: open addressing with linear
 * probing from key % capacity, deletion by chain replacement (each vacated slot is refilled
 * with the LAST entry further along the cluster whose home slot allows the move, and the
 * slot that entry left is refilled the same way, until no entry qualifies), and pruning by
 * one walk over the slots that pops at most one stale frame per visit and re-visits a slot
 * whose entry was deleted (the refill may have moved another entry there).  Table layouts
 * are identical to the reference's for the same operation sequence
 * (tests/test_feature_pool.py compares them slot by slot against the reference's own code). */
#include <string.h>

#include "feature_pool.h"
#include "maveric_hip.h"

#define CAP MV_LOCAL_FEATURE_POOL_CAPACITY
#define NF MV_MAX_LOCAL_FRAMES

/* :24-28 -- the ring and the point are left as they are */
void mv_local_feature_init(mv_local_feature *f) {
    f->word_id = -1;
    f->frame_ptr = 0;
    f->num_frames = 0;
}

/* :30-35 */
void mv_local_feature_init_with_id(mv_local_feature *f, int word_id, int frame_num) {
    f->word_id = word_id;
    f->frame_ptr = 0;
    f->num_frames = 1;
    f->frames[0] = frame_num;
}

/* :37-47: append while the ring has room, else overwrite the oldest and advance */
void mv_local_feature_update(mv_local_feature *f, int frame_num) {
    if (f->num_frames < NF) {
        f->frames[(f->frame_ptr + f->num_frames) % NF] = frame_num;
        f->num_frames++;
        return;
    }
    f->frames[f->frame_ptr] = frame_num;
    f->frame_ptr = (f->frame_ptr + 1) % NF;
}

/* :49-62: drops the oldest frame if it is older than oldest_keep_frame (one per call);
 * true when the feature has no frame left.  A feature already without frames is left as it is:
 * that state exists only after a delete that could not find its key (where the reference exits,
 * mv_local_feature_pool_remove_old's error), and decrementing again would drive num_frames
 * negative -- the next update would index the ring out of bounds (found by the host sanitizer
 * build, tests/test_sanitize.py). */
bool mv_local_feature_remove_old_frame(mv_local_feature *f, int oldest_keep_frame) {
    if (f->word_id == -1) return false;
    if (f->num_frames <= 0) return true;
    if (f->frames[f->frame_ptr] < oldest_keep_frame) {
        f->frame_ptr = (f->frame_ptr + 1) % NF;
        f->num_frames--;
    }
    return f->num_frames == 0;
}

static void entry_clear(mv_lfp_entry *e) { /* init_hash_entry / delete_hash_entry (:70-80) */
    e->key = -1;
    e->is_occupied = false;
    mv_local_feature_init(&e->value);
}

static int home(int key, int capacity) { return key % capacity; } /* hash (:93-95) */

void mv_local_feature_pool_init(mv_local_feature_pool *pool) {
    pool->size = 0;
    pool->capacity = CAP;
    for (int i = 0; i < CAP; i++) entry_clear(&pool->entries[i]);
}

int mv_local_feature_pool_insert(mv_local_feature_pool *pool, int key, const mv_local_feature *value,
                                 mv_local_feature **feature, bool *inserted) {
    *feature = NULL;
    *inserted = false;
    if (key < 0) return MV_ERR_INVALID_ARG; /* the reference would probe from a negative slot */
    if (pool->size >= pool->capacity) return MV_ERR_CAPACITY;
    const int cap = pool->capacity;
    for (int n = 0, s = home(key, cap); n < cap; n++, s = (s + 1) % cap) {
        mv_lfp_entry *e = &pool->entries[s];
        if (e->key == key) { /* present: the existing feature, not inserted */
            *feature = &e->value;
            return MV_OK;
        }
        if (!e->is_occupied) {
            pool->size++;
            e->key = key;
            e->value = *value;
            e->is_occupied = true;
            *feature = &e->value;
            *inserted = true;
            return MV_OK;
        }
    }
    return MV_ERR_CAPACITY; /* unreachable while size < capacity */
}

/* :137-168.  The scan after `hole` runs to the end of the cluster and keeps the last slot
 * whose entry may move back into the hole: before the scan wraps past slot 0, any entry
 * homed at or before the hole; after it wraps, one homed after its own slot but at or
 * before the hole.  Returns the slot finally left empty. */
static int refill_chain(mv_local_feature_pool *pool, int hole) {
    const int cap = pool->capacity;
    int last = hole;
    for (;;) {
        int pick = -1;
        int s = (hole + 1) % cap;
        bool wrapped = s == 0;
        for (int n = 0; n < cap; n++) {
            const mv_lfp_entry *e = &pool->entries[s];
            if (!e->is_occupied) break;
            const int h = home(e->key, cap);
            if (wrapped ? (h > s && h <= hole) : (h <= hole)) pick = s;
            s = (s + 1) % cap;
            if (s == 0) wrapped = true;
        }
        if (pick < 0) break;
        pool->entries[hole] = pool->entries[pick];
        hole = pick;
        last = pick;
    }
    return last;
}

int mv_local_feature_pool_delete(mv_local_feature_pool *pool, int key) {
    if (key < 0) return MV_ERR_INVALID_ARG;
    const int cap = pool->capacity;
    int at = -1;
    for (int n = 0, s = home(key, cap); n < cap; n++, s = (s + 1) % cap) {
        if (!pool->entries[s].is_occupied) return MV_ERR_INVALID_ARG; /* absent (:177-180 exits) */
        if (pool->entries[s].key == key) {
            at = s;
            break;
        }
    }
    if (at < 0) return MV_ERR_INVALID_ARG;
    entry_clear(&pool->entries[refill_chain(pool, at)]);
    pool->size--;
    return MV_OK;
}

/* :258-269.  A delete that cannot find its key (an entry made unreachable by the refill
 * rule, see feature_pool.h) is where the reference exits: stop there and report it. */
int mv_local_feature_pool_remove_old(mv_local_feature_pool *pool, int current_frame_num) {
    const int keep = current_frame_num - NF + 1;
    for (int i = 0; i < pool->capacity; i++) {
        mv_lfp_entry *e = &pool->entries[i];
        if (e->is_occupied && mv_local_feature_remove_old_frame(&e->value, keep)) {
            if (mv_local_feature_pool_delete(pool, e->key) != MV_OK) return MV_ERR_INVALID_ARG;
            i--; /* the refill may have moved another entry into slot i */
        }
    }
    return MV_OK;
}

void mv_local_feature_pool_valid_keys(const mv_local_feature_pool *pool, int *num_keys, int *keys) {
    for (int i = 0; i < pool->capacity; i++)
        if (pool->entries[i].is_occupied) keys[(*num_keys)++] = pool->entries[i].key;
}

float mv_local_feature_pool_load_factor(const mv_local_feature_pool *pool) {
    return (float)pool->size / pool->capacity;
}

int mv_local_feature_pool_check_invariant(const mv_local_feature_pool *pool, int cur_frame) {
    int size = 0;
    for (int i = 0; i < pool->capacity; i++) {
        const mv_lfp_entry *e = &pool->entries[i];
        if (!e->is_occupied) continue;
        size++;
        const mv_local_feature *f = &e->value;
        if (e->key == -1 || f->word_id != e->key || f->num_frames < 1) return MV_ERR_INVALID_ARG;
        int p = f->frame_ptr;
        if (f->frames[p] < cur_frame - NF + 1) return MV_ERR_INVALID_ARG; /* too old */
        for (int j = 1; j < f->num_frames; j++) {                          /* strictly increasing */
            const int q = (p + 1) % NF;
            if (f->frames[q] <= f->frames[p]) return MV_ERR_INVALID_ARG;
            p = q;
        }
    }
    return size == pool->size ? MV_OK : MV_ERR_INVALID_ARG;
}

int mv_local_feature_pool_track_frame(mv_local_feature_pool *pool, int frame_num, int n, const int *word_ids) {
    if (n < 0 || (n > 0 && !word_ids)) return MV_ERR_INVALID_ARG;
    for (int i = 0; i < n; i++) {
        mv_local_feature f;
        memset(&f, 0, sizeof f);
        mv_local_feature_init_with_id(&f, word_ids[i], frame_num);
        mv_local_feature *at;
        bool inserted;
        const int rc = mv_local_feature_pool_insert(pool, word_ids[i], &f, &at, &inserted);
        if (rc != MV_OK) return rc;
        if (!inserted) mv_local_feature_update(at, frame_num);
    }
    return mv_local_feature_pool_remove_old(pool, frame_num);
}
