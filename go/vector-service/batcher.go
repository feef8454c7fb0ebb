package main

import (
	"sync"

	"gorilla-rag/vsearch"
)

// batcher coalesces concurrent /search requests into batched engine calls.
// net/http runs every handler on its own goroutine (main.go:77); each one
// hands its query here and waits. One goroutine per device (lane) makes one
// engine call per turn for the collection of the oldest waiting request,
// with every waiting request of that collection (up to maxBatch): a batch of
// queries streams the corpus once (the MFMA path) instead of once per query.
// While a call runs, new requests queue, so batches grow with the load and a
// lone request waits for nothing. Exact: each request gets the first k of
// the batch's k_max results, and results are totally ordered (score desc,
// row asc). Lanes: a request goes to the lane of its collection's device
// (Engine.Placement; -1 for a row-striped collection), so with collections
// placed on different GPUs (VS_PLACEMENT=collections) their calls run
// concurrently.
type batcher struct {
	eng      *vsearch.Engine
	dim      uint32
	maxBatch int
	mu       sync.Mutex
	lanes    map[int]chan *pending
}

type pending struct {
	coll string
	q    []float32
	k    uint32
	done chan result
}

type result struct {
	hits vsearch.Hits
	err  error
}

// kMFMA: the engine's batched path serves k <= 128; larger k are grouped
// apart so they never move small-k requests off it.
const kMFMA = 128

func newBatcher(eng *vsearch.Engine, dim uint32) *batcher {
	return &batcher{eng: eng, dim: dim, maxBatch: 256, lanes: map[int]chan *pending{}}
}

// lane returns the queue of the device holding coll, starting its goroutine
// on first use.
func (b *batcher) lane(coll string) chan *pending {
	dev, err := b.eng.Placement(coll)
	if err != nil {
		dev = -1
	}
	b.mu.Lock()
	defer b.mu.Unlock()
	ch, ok := b.lanes[dev]
	if !ok {
		ch = make(chan *pending, 4096)
		b.lanes[dev] = ch
		go b.run(ch)
	}
	return ch
}

func (b *batcher) search(coll string, q []float32, k uint32) (vsearch.Hits, error) {
	p := &pending{coll: coll, q: q, k: k, done: make(chan result, 1)}
	b.lane(coll) <- p
	r := <-p.done
	return r.hits, r.err
}

func (b *batcher) run(in chan *pending) {
	var queue []*pending
	for {
		if len(queue) == 0 {
			queue = append(queue, <-in)
		}
		for more := true; more; {
			select {
			case p := <-in:
				queue = append(queue, p)
			default:
				more = false
			}
		}
		head := queue[0]
		var group, rest []*pending
		for _, p := range queue {
			if p.coll == head.coll && (p.k > kMFMA) == (head.k > kMFMA) && len(group) < b.maxBatch {
				group = append(group, p)
			} else {
				rest = append(rest, p)
			}
		}
		queue = rest
		b.execute(group)
	}
}

func (b *batcher) execute(group []*pending) {
	kmax := uint32(1)
	flat := make([]float32, 0, len(group)*int(b.dim))
	for _, p := range group {
		if p.k > kmax {
			kmax = p.k
		}
		flat = append(flat, p.q...)
	}
	hits, err := b.eng.SearchBatch(group[0].coll, flat, b.dim, kmax)
	for i, p := range group {
		if err != nil {
			p.done <- result{err: err}
			continue
		}
		h := hits[i]
		n := int(p.k)
		if n > len(h.Rows) {
			n = len(h.Rows)
		}
		p.done <- result{hits: vsearch.Hits{Rows: h.Rows[:n], Scores: h.Scores[:n]}}
	}
}
