/*
 * ref_pool_harness.c -- drives the reference's OWN local feature pool
 * (include/local_feature_pool.h) and its workload generator (src/local_feature_matching.c:
 * generate_word_ids, srand(0) + rand()), compiled from their sources by oracle/Makefile into
 * oracle/_ref/libmv_ref_pool.so: the reference file is #included below with its main()
 * renamed, so every pool operation and every generated id is the reference's.  Only the
 * frame loop of its main() (:138-171) is restated, to dump the table after each frame.
 * Test infrastructure (tests/test_feature_pool.py); never shipped or measured as product.
 */
#include <setjmp.h>
#include <stdlib.h>
#include <string.h>

/* the reference exit()s where its pool gives up (local_feature_pool.h:179 "Key not found",
 * :298-331 invariant checks): here that returns to the harness entry instead of ending the
 * test process, and the entry reports the frame it happened in */
static jmp_buf ref_jb;
static void ref_exit(int code) {
    (void)code;
    longjmp(ref_jb, 1);
}
#define exit(x) ref_exit(x)
#define main ref_lfm_main
#include "local_feature_matching.c"
#undef main
#undef exit

#define REF_POOL_WORDS 13 /* per slot: key, occupied, word_id, frame_ptr, num_frames, frames[8] */

int ref_pool_sizeof(void) { return (int)sizeof(LocalFeaturePool); }
int ref_pool_capacity(void) { return LOCAL_FEATURE_POOL_CAPACITY; }

static void dump(const LocalFeaturePool *pool, int *t) {
    for (int i = 0; i < pool->capacity; i++) {
        const HashEntry *e = &pool->entries[i];
        t[0] = e->key;
        t[1] = e->is_occupied ? 1 : 0;
        t[2] = e->value.word_id;
        t[3] = e->value.frame_ptr;
        t[4] = e->value.num_frames;
        for (int j = 0; j < MAX_LOCAL_FRAMES; j++) t[5 + j] = e->value.frames[j];
        t += REF_POOL_WORDS;
    }
}

/* main()'s loop body for one frame (:153-164) on the given ids; the local feature is zeroed
 * first (main leaves its unused ring slots as stack garbage) */
static void one_frame(LocalFeaturePool *pool, int frame, int n, const int *ids) {
    for (int i = 0; i < n; i++) {
        LocalFeature feature;
        memset(&feature, 0, sizeof feature);
        init_local_feature_with_id(&feature, ids[i], frame);
        LocalFeaturePoolInsertResult result = local_feature_pool_insert(pool, ids[i], feature);
        if (!result.inserted) update_local_feature(result.feature, frame);
    }
    local_feature_pool_remove_old(pool, frame);
    local_feature_pool_check_invariant(pool, frame, false); /* exits on a violation */
}

/* the reference workload: num_frames frames of nfeat ids from generate_word_ids (srand(0));
 * ids_out [num_frames][nfeat], table_out [num_frames][capacity][13], size_out [num_frames] */
int ref_pool_run(int num_frames, int nfeat, int *ids_out, int *table_out, int *size_out) {
    static LocalFeaturePool pool;
    static volatile int frame;
    memset(&pool, 0, sizeof pool);
    srand(0);
    init_local_feature_pool(&pool);
    if (setjmp(ref_jb)) return frame;
    for (frame = 0; frame < num_frames; frame++) {
        int *ids = ids_out + (long)frame * nfeat;
        generate_word_ids(&pool, nfeat, ids);
        one_frame(&pool, frame, nfeat, ids);
        dump(&pool, table_out + (long)frame * pool.capacity * REF_POOL_WORDS);
        size_out[frame] = pool.size;
    }
    return num_frames;
}

/* the same loop on caller-chosen ids (distinct within a frame, >= 0, pool never full).
 * Returns the number of frames completed: num_frames, or the frame in which the reference
 * exit()ed (its tables past that frame are not written). */
int ref_pool_replay(int num_frames, const int *nfeat, const int *ids, int *table_out, int *size_out) {
    static LocalFeaturePool pool;
    static volatile int frame;
    memset(&pool, 0, sizeof pool);
    init_local_feature_pool(&pool);
    if (setjmp(ref_jb)) return frame;
    for (frame = 0; frame < num_frames; frame++) {
        one_frame(&pool, frame, nfeat[frame], ids);
        ids += nfeat[frame];
        dump(&pool, table_out + (long)frame * pool.capacity * REF_POOL_WORDS);
        size_out[frame] = pool.size;
    }
    return num_frames;
}
