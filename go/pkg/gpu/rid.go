package gpu

import (
	"context"
	"sync"
	"sync/atomic"
	"time"

	"github.com/golang/geo/s2"
	dsserr "github.com/interuss/dss/pkg/errors"
	dssmodels "github.com/interuss/dss/pkg/models"
	ridmodels "github.com/interuss/dss/pkg/rid/models"
	"github.com/interuss/dss/pkg/rid/repos"
)

// RIDTransactor decorates the reference's CockroachDB repos.Transactor
// (pkg/rid/cockroach/store.go): writes and point reads go to CRDB, while
// SearchISAs, SearchSubscriptions, SearchSubscriptionsByOwner and
// MaxSubscriptionCountInCellsByOwner run on GPU mirrors of the
// identification_service_areas / subscriptions tables' cells, time and
// owner columns, and UpdateNotificationIdxsInCells finds its subscriptions
// on the mirror (CRDB runs only the UPDATE ... RETURNING of their counters,
// through the hook of go/patches/0002).  Writes made inside InTxnRetrier
// reach the mirrors once the transaction has committed; inside it, the
// fan-out overlays the transaction's own subscription writes.
type RIDTransactor struct {
	repos.Transactor
	// Now is the store clock (cockroach.DefaultClock in the reference).
	Now func() time.Time

	isas, subs *Mirror
	mu         sync.RWMutex
	// writeMu serialises the writers (as SCDTransactor.writeMu does): every
	// write and every notification fan-out read of the subscriptions mirror
	// runs under it, from before the write / read to the mirrors' apply, so
	// a subscription committed to CRDB is on the mirror before any later
	// fan-out reads it.  Autocommit methods hold it for their one statement;
	// a transaction run by InTxnRetrier from its first write or fan-out until
	// its commit is applied.  (A transaction must not call the transactor's
	// autocommit methods after its own first write: the reference's
	// application never does -- InsertISA's transaction calls only those.)
	writeMu    sync.Mutex
	isaRows    map[dssmodels.ID]*ridmodels.IdentificationServiceArea
	subRows    map[dssmodels.ID]*ridmodels.Subscription
	invalid    int32 // atomic: 1 after a failed apply of committed writes (searches then run on CRDB)
}

// Invalid reports whether the mirrors fell behind CRDB.
func (t *RIDTransactor) Invalid() bool { return atomic.LoadInt32(&t.invalid) != 0 }

// applyCommitted mirrors writes CRDB has already committed: a failure cannot
// undo them, so it marks the mirrors invalid instead of failing the call.
func (t *RIDTransactor) applyCommitted(w *ridWrites) {
	if err := t.apply(w); err != nil {
		atomic.StoreInt32(&t.invalid, 1)
	}
}

// NewRIDTransactor builds the mirrors from the tables' current rows.
func NewRIDTransactor(inner repos.Transactor, isas []*ridmodels.IdentificationServiceArea, subs []*ridmodels.Subscription) (*RIDTransactor, error) {
	t := &RIDTransactor{Transactor: inner, Now: time.Now,
		isaRows: map[dssmodels.ID]*ridmodels.IdentificationServiceArea{}, subRows: map[dssmodels.ID]*ridmodels.Subscription{}}
	var err error
	if t.isas, err = NewMirror(false); err != nil {
		return nil, err
	}
	if t.subs, err = NewMirror(true); err != nil {
		return nil, err
	}
	w := newRIDWrites()
	for _, i := range isas {
		w.isas[i.ID] = i
	}
	for _, s := range subs {
		w.subs[s.ID] = s
	}
	if err := t.apply(w); err != nil {
		return nil, err
	}
	return t, nil
}

// RID rows have no altitude filter in any search (identification_service_area.go:166-197).
func isaRow(i *ridmodels.IdentificationServiceArea) Row {
	return Row{Key: i.ID.String(), Cells: i.Cells, AltLo: negInf, AltHi: posInf,
		T0: usOrNull(i.StartTime, timeNullStart), T1: usOrNull(i.EndTime, timeNullStored), Owner: i.Owner.String()}
}

func ridSubRow(s *ridmodels.Subscription) Row {
	return Row{Key: s.ID.String(), Cells: s.Cells, AltLo: negInf, AltHi: posInf,
		T0: usOrNull(s.StartTime, timeNullStart), T1: usOrNull(s.EndTime, timeNullStored), Owner: s.Owner.String()}
}

// ridWrites is a set of committed row changes (nil value: deleted).
type ridWrites struct {
	isas map[dssmodels.ID]*ridmodels.IdentificationServiceArea
	subs map[dssmodels.ID]*ridmodels.Subscription
}

func newRIDWrites() *ridWrites {
	return &ridWrites{isas: map[dssmodels.ID]*ridmodels.IdentificationServiceArea{},
		subs: map[dssmodels.ID]*ridmodels.Subscription{}}
}

func (t *RIDTransactor) apply(w *ridWrites) error {
	t.mu.Lock()
	defer t.mu.Unlock()
	var rows []Row
	var dels []string
	for id, i := range w.isas {
		if i == nil {
			dels = append(dels, id.String())
			delete(t.isaRows, id)
		} else {
			rows = append(rows, isaRow(i))
			t.isaRows[id] = i
		}
	}
	if err := t.isas.Upsert(rows); err != nil {
		return err
	}
	if err := t.isas.Delete(dels); err != nil {
		return err
	}
	rows, dels = rows[:0], dels[:0]
	for id, s := range w.subs {
		if s == nil {
			dels = append(dels, id.String())
			delete(t.subRows, id)
		} else {
			rows = append(rows, ridSubRow(s))
			t.subRows[id] = s
		}
	}
	if err := t.subs.Upsert(rows); err != nil {
		return err
	}
	return t.subs.Delete(dels)
}

// InTxnRetrier runs f on a recording repo; the last attempt's writes are
// mirrored once the inner retrier reports the transaction committed.
func (t *RIDTransactor) InTxnRetrier(ctx context.Context, f func(repo repos.Repository) error) error {
	var w *ridWrites
	lk := &txLock{mu: &t.writeMu}
	defer lk.unlock() // after the apply below
	err := t.Transactor.InTxnRetrier(ctx, func(repo repos.Repository) error {
		w = newRIDWrites() // a retried attempt starts over
		return f(&ridRepo{Repository: repo, w: w, t: t, lk: lk})
	})
	if err != nil || w == nil {
		return err
	}
	t.applyCommitted(w)
	return nil
}

// txLock is a transaction's hold on the write lock: taken once, at its first
// write or fan-out read, released after its commit's apply.
type txLock struct {
	mu     *sync.Mutex
	locked bool
}

func (l *txLock) lock() {
	if !l.locked {
		l.mu.Lock()
		l.locked = true
	}
}

func (l *txLock) unlock() {
	if l.locked {
		l.locked = false
		l.mu.Unlock()
	}
}

// ---- the transactor's own (autocommit) repository methods ---------------

func (t *RIDTransactor) InsertISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.InsertISA(ctx, isa)
	if err == nil && res != nil {
		w := newRIDWrites()
		w.isas[res.ID] = res
		t.applyCommitted(w)
	}
	return res, err
}

func (t *RIDTransactor) UpdateISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.UpdateISA(ctx, isa)
	if err == nil && res != nil {
		w := newRIDWrites()
		w.isas[res.ID] = res
		t.applyCommitted(w)
	}
	return res, err
}

func (t *RIDTransactor) DeleteISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.DeleteISA(ctx, isa)
	if err == nil {
		w := newRIDWrites()
		w.isas[isa.ID] = nil
		t.applyCommitted(w)
	}
	return res, err
}

func (t *RIDTransactor) InsertSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.InsertSubscription(ctx, sub)
	if err == nil && res != nil {
		w := newRIDWrites()
		w.subs[res.ID] = res
		t.applyCommitted(w)
	}
	return res, err
}

func (t *RIDTransactor) UpdateSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.UpdateSubscription(ctx, sub)
	if err == nil && res != nil {
		w := newRIDWrites()
		w.subs[res.ID] = res
		t.applyCommitted(w)
	}
	return res, err
}

func (t *RIDTransactor) DeleteSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	res, err := t.Transactor.DeleteSubscription(ctx, sub)
	if err == nil {
		w := newRIDWrites()
		w.subs[sub.ID] = nil
		t.applyCommitted(w)
	}
	return res, err
}

// idUpdater is the reference subscription store with the hook of
// go/patches/0002-scd-rid-gpu-store-hooks.patch.
type idUpdater interface {
	UpdateNotificationIdxsByIDs(ctx context.Context, ids []dssmodels.ID) ([]*ridmodels.Subscription, error)
}

// notifyIDs is UpdateNotificationIdxsInCells' `cells && $1 AND ends_at >=
// now` (subscriptions.go:204-219) on the subscriptions mirror, with the
// subscription writes w of the calling transaction (nil outside one)
// overlaid.  ok = false: the mirror cannot answer (invalid).
func (t *RIDTransactor) notifyIDs(cells s2.CellUnion, w *ridWrites) (ids []dssmodels.ID, ok bool, err error) {
	if t.Invalid() {
		return nil, false, nil
	}
	if len(cells) == 0 {
		return nil, true, nil // cells && '{}' holds for no row
	}
	q := Query{Cells: cells, AltLo: negInf, AltHi: posInf, TLo: usOf(t.Now()), THi: timeNullEndQ}
	t.mu.RLock()
	keys, err := t.subs.Search([]Query{q})
	t.mu.RUnlock()
	if err != nil {
		return nil, false, err
	}
	for _, k := range keys[0] {
		id := dssmodels.ID(k)
		if w != nil {
			if _, written := w.subs[id]; written {
				continue // this transaction's version decides
			}
		}
		ids = append(ids, id)
	}
	if w != nil {
		for id, sub := range w.subs {
			if sub != nil && ridSubRow(sub).Matches(q) {
				ids = append(ids, id)
			}
		}
	}
	return ids, true, nil
}

// UpdateNotificationIdxsInCells: the subscriptions are found on the mirror
// (notifyIDs); CRDB runs only the UPDATE ... WHERE id = ANY($ids) ...
// RETURNING of their counters (UpdateNotificationIdxsByIDs, patch 0002).
// The returned rows refresh the cache.
func (t *RIDTransactor) UpdateNotificationIdxsInCells(ctx context.Context, cells s2.CellUnion) ([]*ridmodels.Subscription, error) {
	t.writeMu.Lock()
	defer t.writeMu.Unlock()
	var res []*ridmodels.Subscription
	var err error
	ids, ok, err := t.notifyIDs(cells, nil)
	if err != nil {
		return nil, err
	}
	if u, hooked := t.Transactor.(idUpdater); hooked && ok {
		res, err = u.UpdateNotificationIdxsByIDs(ctx, ids)
	} else {
		res, err = t.Transactor.UpdateNotificationIdxsInCells(ctx, cells)
	}
	if err == nil && len(res) > 0 {
		w := newRIDWrites()
		for _, s := range res {
			w.subs[s.ID] = s
		}
		t.applyCommitted(w)
	}
	return res, err
}

// MaxSubscriptionCountInCellsByOwner replaces the reference's
// (pkg/rid/cockroach/subscriptions.go:83-116; its TODO at :87-89 asks for
// this count to be kept in memory): the subscriptions mirror answers it
// (Mirror.MaxCount, dssg_store_max_subscription_count).  The caller
// (application/subscription.go:69) runs it outside a transaction, as the
// reference does.
func (t *RIDTransactor) MaxSubscriptionCountInCellsByOwner(ctx context.Context, cells s2.CellUnion, owner dssmodels.Owner) (int, error) {
	if t.Invalid() {
		return t.Transactor.MaxSubscriptionCountInCellsByOwner(ctx, cells, owner)
	}
	t.mu.RLock()
	defer t.mu.RUnlock()
	return t.subs.MaxCount(cells, owner.String(), usOf(t.Now()))
}

// SearchISAs replaces (*ISAStore).SearchISAs
// (pkg/rid/cockroach/identification_service_area.go:166-197):
//   ends_at >= earliest AND COALESCE(starts_at <= latest, true) AND cells && cells.
func (t *RIDTransactor) SearchISAs(ctx context.Context, cells s2.CellUnion, earliest *time.Time, latest *time.Time) ([]*ridmodels.IdentificationServiceArea, error) {
	if len(cells) == 0 {
		return nil, dsserr.BadRequest("missing cell IDs for query")
	}
	if earliest == nil {
		return nil, dsserr.Internal("must call with an earliest start time.")
	}
	if t.Invalid() {
		return t.Transactor.SearchISAs(ctx, cells, earliest, latest)
	}
	q := Query{Cells: cells, AltLo: negInf, AltHi: posInf, TLo: usOf(*earliest),
		THi: usOrNull(latest, timeNullEndQ)}
	t.mu.RLock() // across the search and the lookup: no apply lands in between
	defer t.mu.RUnlock()
	keys, err := t.isas.Search([]Query{q})
	if err != nil {
		return nil, err
	}
	out := make([]*ridmodels.IdentificationServiceArea, 0, len(keys[0]))
	for _, k := range keys[0] {
		if i, ok := t.isaRows[dssmodels.ID(k)]; ok {
			c := *i
			out = append(out, &c)
		}
	}
	return out, nil
}

func (t *RIDTransactor) searchSubs(cells s2.CellUnion, owner string) ([]*ridmodels.Subscription, error) {
	if len(cells) == 0 {
		return nil, dsserr.BadRequest("no location provided")
	}
	q := Query{Cells: cells, AltLo: negInf, AltHi: posInf, TLo: usOf(t.Now()), THi: timeNullEndQ,
		Owner: owner}
	t.mu.RLock() // across the search and the lookup: no apply lands in between
	defer t.mu.RUnlock()
	keys, err := t.subs.Search([]Query{q})
	if err != nil {
		return nil, err
	}
	out := make([]*ridmodels.Subscription, 0, len(keys[0]))
	for _, k := range keys[0] {
		if s, ok := t.subRows[dssmodels.ID(k)]; ok {
			c := *s
			out = append(out, &c)
		}
	}
	return out, nil
}

// SearchSubscriptions replaces (*SubscriptionStore).SearchSubscriptions
// (pkg/rid/cockroach/subscriptions.go:222-244): cells && cells AND ends_at >= now.
func (t *RIDTransactor) SearchSubscriptions(ctx context.Context, cells s2.CellUnion) ([]*ridmodels.Subscription, error) {
	if t.Invalid() {
		return t.Transactor.SearchSubscriptions(ctx, cells)
	}
	return t.searchSubs(cells, "")
}

// SearchSubscriptionsByOwner replaces (*SubscriptionStore).SearchSubscriptionsByOwner
// (pkg/rid/cockroach/subscriptions.go:247-273): the same AND owner = $owner.
func (t *RIDTransactor) SearchSubscriptionsByOwner(ctx context.Context, cells s2.CellUnion, owner dssmodels.Owner) ([]*ridmodels.Subscription, error) {
	if t.Invalid() {
		return t.Transactor.SearchSubscriptionsByOwner(ctx, cells, owner)
	}
	return t.searchSubs(cells, owner.String())
}

// ridRepo is the repository InTxnRetrier hands to f: CRDB in the
// transaction, with writes recorded for the mirrors.
type ridRepo struct {
	repos.Repository
	w  *ridWrites
	t  *RIDTransactor
	lk *txLock
}

func (r *ridRepo) InsertISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	r.lk.lock()
	res, err := r.Repository.InsertISA(ctx, isa)
	if err == nil && res != nil {
		r.w.isas[res.ID] = res
	}
	return res, err
}

func (r *ridRepo) UpdateISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	r.lk.lock()
	res, err := r.Repository.UpdateISA(ctx, isa)
	if err == nil && res != nil {
		r.w.isas[res.ID] = res
	}
	return res, err
}

func (r *ridRepo) DeleteISA(ctx context.Context, isa *ridmodels.IdentificationServiceArea) (*ridmodels.IdentificationServiceArea, error) {
	r.lk.lock()
	res, err := r.Repository.DeleteISA(ctx, isa)
	if err == nil {
		r.w.isas[isa.ID] = nil
	}
	return res, err
}

func (r *ridRepo) InsertSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	r.lk.lock()
	res, err := r.Repository.InsertSubscription(ctx, sub)
	if err == nil && res != nil {
		r.w.subs[res.ID] = res
	}
	return res, err
}

func (r *ridRepo) UpdateSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	r.lk.lock()
	res, err := r.Repository.UpdateSubscription(ctx, sub)
	if err == nil && res != nil {
		r.w.subs[res.ID] = res
	}
	return res, err
}

func (r *ridRepo) DeleteSubscription(ctx context.Context, sub *ridmodels.Subscription) (*ridmodels.Subscription, error) {
	r.lk.lock()
	res, err := r.Repository.DeleteSubscription(ctx, sub)
	if err == nil {
		r.w.subs[sub.ID] = nil
	}
	return res, err
}

// UpdateNotificationIdxsInCells inside the transaction (application/isa.go:69
// and its insert / delete siblings): the subscription ids from the mirror
// with this transaction's own subscription writes overlaid, the UPDATE ...
// RETURNING on the transaction.
func (r *ridRepo) UpdateNotificationIdxsInCells(ctx context.Context, cells s2.CellUnion) ([]*ridmodels.Subscription, error) {
	r.lk.lock()
	var res []*ridmodels.Subscription
	ids, ok, err := r.t.notifyIDs(cells, r.w)
	if err != nil {
		return nil, err
	}
	if u, hooked := r.Repository.(idUpdater); hooked && ok {
		res, err = u.UpdateNotificationIdxsByIDs(ctx, ids)
	} else {
		res, err = r.Repository.UpdateNotificationIdxsInCells(ctx, cells)
	}
	if err == nil {
		for _, s := range res {
			r.w.subs[s.ID] = s
		}
	}
	return res, err
}
