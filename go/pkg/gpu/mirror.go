package gpu

/*
#include "dssgpu.h"
*/
import "C"

import (
	"fmt"
	"sync"
	"unsafe"

	"github.com/golang/geo/s2"
)

// Row is the 4D part of one stored entity (an operation, ISA or
// subscription): what the CRDB schema keeps in the cells / altitude / time /
// owner columns (pkg/scd/store/cockroach/store.go:120-147,
// pkg/rid/cockroach/store.go:122-151).
type Row struct {
	Key          string // the entity id
	Cells        s2.CellUnion
	AltLo, AltHi float32 // NULL: -Inf / +Inf
	T0, T1       int64   // unix us; NULL start: math.MinInt64, NULL ends_at: math.MinInt64 (never matches)
	Owner        string
}

// Query is one search volume, already folded into the ABI's bounds
// (e.t1 >= TLo AND e.t0 <= THi AND the altitude overlap AND owner).
type Query struct {
	Cells        s2.CellUnion
	AltLo, AltHi float32
	TLo, THi     int64
	Owner        string // "" = any owner
}

// Mirror is the GPU-resident copy of one table's 4D columns, behind
// dssg_store (base + delta indexes with tombstones, dssgpu.h).  Writes are
// serialised by the mirror; searches run concurrently, each on its own
// context from the pool.
type Mirror struct {
	mu        sync.RWMutex
	st        *C.dssg_store
	withOwner bool
	ids       map[string]uint32 // key -> dense id
	keys      []string          // dense id -> key ("" = free)
	free      []uint32
	owners    map[string]int32
}

// NewMirror creates an empty mirror; withOwner keeps owner ids for
// owner-filtered searches (RID SearchSubscriptionsByOwner).
func NewMirror(withOwner bool) (*Mirror, error) {
	c, err := getCtx()
	if err != nil {
		return nil, err
	}
	defer putCtx(c)
	m := &Mirror{withOwner: withOwner, ids: map[string]uint32{}, owners: map[string]int32{}}
	wo := C.int32_t(0)
	if withOwner {
		wo = 1
	}
	if rc := C.dssg_store_create(c.c, wo, &m.st); rc != C.DSSG_OK {
		return nil, c.err("dssg_store_create", rc)
	}
	return m, nil
}

// Close frees the device copy.
func (m *Mirror) Close() {
	m.mu.Lock()
	defer m.mu.Unlock()
	if m.st != nil {
		C.dssg_store_free(m.st)
		m.st = nil
	}
}

func (m *Mirror) ownerID(o string) int32 {
	if o == "" {
		return -1
	}
	id, ok := m.owners[o]
	if !ok {
		id = int32(len(m.owners))
		m.owners[o] = id
	}
	return id
}

// Upsert writes rows (insert or replace by key), as one dssg_store_upsert.
func (m *Mirror) Upsert(rows []Row) error {
	if len(rows) == 0 {
		return nil
	}
	m.mu.Lock()
	defer m.mu.Unlock()
	c, err := getCtx()
	if err != nil {
		return err
	}
	defer putCtx(c)
	n := len(rows)
	ids := make([]C.uint32_t, n)
	offs := make([]C.int64_t, n+1)
	lo, hi := make([]C.float, n), make([]C.float, n)
	t0, t1 := make([]C.int64_t, n), make([]C.int64_t, n)
	own := make([]C.int32_t, n)
	for i, r := range rows {
		id, ok := m.ids[r.Key]
		if !ok {
			if k := len(m.free); k > 0 {
				id = m.free[k-1]
				m.free = m.free[:k-1]
				m.keys[id] = r.Key
			} else {
				id = uint32(len(m.keys))
				m.keys = append(m.keys, r.Key)
			}
			m.ids[r.Key] = id
		}
		ids[i] = C.uint32_t(id)
		offs[i+1] = offs[i] + C.int64_t(len(r.Cells))
		lo[i], hi[i] = C.float(r.AltLo), C.float(r.AltHi)
		t0[i], t1[i] = C.int64_t(r.T0), C.int64_t(r.T1)
		own[i] = C.int32_t(m.ownerID(r.Owner))
	}
	cells := make([]uint64, int(offs[n])+1)
	for i, r := range rows {
		for k, cid := range r.Cells {
			cells[int(offs[i])+k] = uint64(cid)
		}
	}
	var ownp *C.int32_t
	if m.withOwner {
		ownp = &own[0]
	}
	if rc := C.dssg_store_upsert(c.c, m.st, C.int64_t(n), &ids[0], &offs[0], (*C.uint64_t)(unsafe.Pointer(&cells[0])),
		&lo[0], &hi[0], &t0[0], &t1[0], ownp); rc != C.DSSG_OK {
		return c.err("dssg_store_upsert", rc)
	}
	return nil
}

// Delete removes keys (unknown keys are ignored).
func (m *Mirror) Delete(keys []string) error {
	m.mu.Lock()
	defer m.mu.Unlock()
	ids := make([]C.uint32_t, 0, len(keys))
	for _, k := range keys {
		if id, ok := m.ids[k]; ok {
			ids = append(ids, C.uint32_t(id))
			delete(m.ids, k)
			m.keys[id] = ""
			m.free = append(m.free, id)
		}
	}
	if len(ids) == 0 {
		return nil
	}
	c, err := getCtx()
	if err != nil {
		return err
	}
	defer putCtx(c)
	found := make([]C.int32_t, len(ids))
	if rc := C.dssg_store_delete(c.c, m.st, C.int64_t(len(ids)), &ids[0], &found[0]); rc != C.DSSG_OK {
		return c.err("dssg_store_delete", rc)
	}
	return nil
}

// Search runs a batch of queries; result i holds the keys matching query i
// (each once: the SQL DISTINCT / && semantics), in key-id order.  A query
// filtered by an owner that has no row in the mirror matches nothing
// (`subscriptions.owner = $2`, pkg/rid/cockroach/subscriptions.go:245-273)
// and is answered here, never sent: the engine reads a negative owner as
// "any owner" (dssgpu.h), so no sentinel id may stand for it.
func (m *Mirror) Search(qs []Query) ([][]string, error) {
	out := make([][]string, len(qs))
	if len(qs) == 0 {
		return out, nil
	}
	m.mu.RLock()
	defer m.mu.RUnlock()
	sent := make([]int, 0, len(qs)) // engine query k = qs[sent[k]]
	own := make([]C.int32_t, 0, len(qs))
	for i, q := range qs {
		o := C.int32_t(-1)
		if q.Owner != "" {
			id, ok := m.owners[q.Owner]
			if !ok {
				continue // no rows of this owner: empty result
			}
			o = C.int32_t(id)
		}
		sent = append(sent, i)
		own = append(own, o)
	}
	n := len(sent)
	if n == 0 {
		return out, nil
	}
	c, err := getCtx()
	if err != nil {
		return nil, err
	}
	defer putCtx(c)
	offs := make([]C.int64_t, n+1)
	lo, hi := make([]C.float, n), make([]C.float, n)
	tlo, thi := make([]C.int64_t, n), make([]C.int64_t, n)
	for k, i := range sent {
		q := qs[i]
		offs[k+1] = offs[k] + C.int64_t(len(q.Cells))
		lo[k], hi[k] = C.float(q.AltLo), C.float(q.AltHi)
		tlo[k], thi[k] = C.int64_t(q.TLo), C.int64_t(q.THi)
	}
	cells := make([]uint64, int(offs[n])+1)
	for k, i := range sent {
		for j, cid := range qs[i].Cells {
			cells[int(offs[k])+j] = uint64(cid)
		}
	}
	var ownp *C.int32_t
	if m.withOwner {
		ownp = &own[0]
	}
	pq, pe := make([]uint32, 1024), make([]uint32, 1024)
	for {
		var needed C.int64_t
		rc := C.dssg_store_search(c.c, m.st, C.int64_t(n), &offs[0], (*C.uint64_t)(unsafe.Pointer(&cells[0])), &lo[0],
			&hi[0], &tlo[0], &thi[0], ownp, (*C.uint32_t)(unsafe.Pointer(&pq[0])),
			(*C.uint32_t)(unsafe.Pointer(&pe[0])), C.int64_t(len(pq)), &needed)
		if rc == C.DSSG_ERR_CAPACITY {
			pq, pe = make([]uint32, int(needed)+1), make([]uint32, int(needed)+1)
			continue
		}
		if rc != C.DSSG_OK {
			return nil, c.err("dssg_store_search", rc)
		}
		for k := 0; k < int(needed); k++ {
			if int(pe[k]) >= len(m.keys) || m.keys[pe[k]] == "" {
				return nil, fmt.Errorf("dssg_store_search: id %d not live", pe[k])
			}
			i := sent[pq[k]]
			out[i] = append(out[i], m.keys[pe[k]])
		}
		return out, nil
	}
}

// MaxCount is RID MaxSubscriptionCountInCellsByOwner
// (pkg/rid/cockroach/subscriptions.go:83-116) over the mirror's live rows
// (dssg_store_max_subscription_count): the most rows of owner with ends_at
// >= now posted in any one of cells, repeats of a cell in a row's array
// counted (`unnest(cells)`), 0 when none (IFNULL(MAX(..), 0)).  An owner with
// no row in the mirror has 0 everywhere and is answered here.
func (m *Mirror) MaxCount(cells s2.CellUnion, owner string, now int64) (int, error) {
	if !m.withOwner {
		return 0, fmt.Errorf("MaxCount on a mirror without owners")
	}
	m.mu.RLock()
	defer m.mu.RUnlock()
	id, ok := m.owners[owner]
	if !ok || len(cells) == 0 {
		return 0, nil
	}
	c, err := getCtx()
	if err != nil {
		return 0, err
	}
	defer putCtx(c)
	offs := []C.int64_t{0, C.int64_t(len(cells))}
	own := C.int32_t(id)
	var count C.int64_t
	if rc := C.dssg_store_max_subscription_count(c.c, m.st, 1, &offs[0], cellsPtr(cells), &own, C.int64_t(now),
		&count); rc != C.DSSG_OK {
		return 0, c.err("dssg_store_max_subscription_count", rc)
	}
	return int(count), nil
}

// Len is the number of live rows.
func (m *Mirror) Len() int {
	m.mu.RLock()
	defer m.mu.RUnlock()
	return len(m.ids)
}

// Matches reports whether row r satisfies query q on the host: the ABI's
// predicate (dssgpu.h dssg_search) with the same NULL sentinels -- for the few
// rows a transaction has written but not committed (read-your-writes).
func (r Row) Matches(q Query) bool {
	if !(r.T1 >= q.TLo && r.T0 <= q.THi && r.AltHi >= q.AltLo && r.AltLo <= q.AltHi) {
		return false
	}
	if q.Owner != "" && r.Owner != q.Owner {
		return false
	}
	set := make(map[s2.CellID]struct{}, len(r.Cells))
	for _, c := range r.Cells {
		set[c] = struct{}{}
	}
	for _, c := range q.Cells {
		if _, ok := set[c]; ok {
			return true
		}
	}
	return false
}
