/*
 * mvx_internal.h -- declarations shared by libmvx.so's C sources (not part
 * of the drop-in surface; that is include/mvx_coll.h).
 */
#ifndef MVX_INTERNAL_H
#define MVX_INTERNAL_H

#include <stddef.h>

/* mvx_host.c */
#define MVX_BUF_PAGEABLE 0   /* host memory the DMA engines cannot address */
#define MVX_BUF_PINNED   1   /* page-locked host memory */
#define MVX_BUF_DEVICE   2   /* device or managed memory */
int mvx_buf_kind(const void *p);   /* one pointer-attribute query */
int mvx_host_pinned(const void *p);
void mvx_pcopy(void *dst, const void *src, size_t bytes);
int mvx_copy_threads(void);

#endif
