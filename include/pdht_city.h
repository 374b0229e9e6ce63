/*
 * pdht_city.h -- drop-in for pdht's city.h + citycrc.h (scalar, host).
 *
 * Same symbols, same signatures, same uint128 layout as
 *   /root/reference/libpdht/city.h:54-84    (CityHash64*, CityHash128*)
 *   /root/reference/libpdht/citycrc.h:39-46 (CityHashCrc128*, CityHashCrc256)
 * so a pdht build can replace `#include <city.h>` by this header and link
 * libpdht_hip.so instead of compiling city.c.  Unlike the reference, the CRC
 * variants are always exported (the reference only has them when compiled
 * with -msse4.2, city.c:402); results are identical either way.
 *
 * These are single-key CPU functions (a GPU launch costs microseconds, a
 * key costs nanoseconds).  Batches go through pdht_hip.h.
 */
#ifndef PDHT_CITY_H_
#define PDHT_CITY_H_

#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef CITY_HASH_H_ /* coexist with a reference city.h already included */
typedef uint8_t uint8;
typedef uint32_t uint32;
typedef uint64_t uint64;

typedef struct _uint128 uint128; /* city.h:58-65 */
struct _uint128 {
  uint64 first;  /* low 64 bits  */
  uint64 second; /* high 64 bits */
};
#define Uint128Low64(x) (x).first
#define Uint128High64(x) (x).second
#endif

/* city.h:68 */
uint64 CityHash64(const char *buf, size_t len);
/* city.h:72 */
uint64 CityHash64WithSeed(const char *buf, size_t len, uint64 seed);
/* city.h:76-77 */
uint64 CityHash64WithSeeds(const char *buf, size_t len, uint64 seed0, uint64 seed1);
/* city.h:80 */
uint128 CityHash128(const char *s, size_t len);
/* city.h:84 */
uint128 CityHash128WithSeed(const char *s, size_t len, uint128 seed);
/* citycrc.h:39 */
uint128 CityHashCrc128(const char *s, size_t len);
/* citycrc.h:43 */
uint128 CityHashCrc128WithSeed(const char *s, size_t len, uint128 seed);
/* citycrc.h:46 */
void CityHashCrc256(const char *s, size_t len, uint64 *result);

/* Exported (non-static) by the reference city.c although city.h does not
 * declare them (city.c:173, :190); kept for link-level parity. */
uint128 WeakHashLen32WithSeeds6(uint64 w, uint64 x, uint64 y, uint64 z, uint64 a, uint64 b);
uint128 WeakHashLen32WithSeeds(const char *s, uint64 a, uint64 b);

#ifdef __cplusplus
}
#endif
#endif /* PDHT_CITY_H_ */
