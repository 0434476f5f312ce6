package io.sesam.dukemicroservice.gpu;

import java.util.ArrayList;
import java.util.Collection;
import java.util.List;

import no.priv.garshol.duke.Configuration;
import no.priv.garshol.duke.Processor;
import no.priv.garshol.duke.Record;
import no.priv.garshol.duke.matchers.MatchListener;

/**
 * Processor whose matching loop runs on the GPU (Duke 1.2 Processor.deduplicate, called at
 * App.java:1005 / 1159).  One batch: batchReady, index + commit (dk_upsert; dk_upsert_transient
 * while indexing is disabled, App.java:1130-1132), dk_match, the callbacks replayed on this
 * thread in Duke's order (per query record in batch order its matches / matchesPerhaps in
 * candidate order, or noMatchFor), batchDone.  Mirrors dukehip/processor.py GpuProcessor.
 */
public class GpuProcessor extends Processor {
    private final GpuBlockingDatabase db;
    private final List<MatchListener> listeners = new ArrayList<>();

    public GpuProcessor(Configuration config, GpuBlockingDatabase db) {
        super(config, false);
        this.db = db;
    }

    @Override
    public void addMatchListener(MatchListener listener) {
        super.addMatchListener(listener);
        listeners.add(listener);
    }

    @Override
    public void deduplicate(Collection<Record> records) {
        List<Record> batch = new ArrayList<>(records);
        for (MatchListener l : listeners) l.batchReady(batch.size());
        // records given to Database.index() beforehand (the deleted records of
        // App.java:988-1001, 1121-1137) are committed together with the batch
        List<Record> pending = db.takePending();
        List<Record> all = new ArrayList<>(pending);
        all.addAll(batch);
        int[] allRows = db.indexBatch(all, db.indexingIsDisabled());
        int[] rows = new int[batch.size()];
        System.arraycopy(allRows, pending.size(), rows, 0, rows.length);
        long res = DukeHip.match(db.ctx(), rows);
        try {
            long[] first = DukeHip.resultFirst(res);
            int[] cand = DukeHip.resultCandidate(res);
            double[] prob = DukeHip.resultProb(res);
            byte[] kind = DukeHip.resultKind(res);
            for (int i = 0; i < batch.size(); i++) {
                Record r1 = batch.get(i);
                if (first[i] == first[i + 1]) {
                    for (MatchListener l : listeners) l.noMatchFor(r1);
                    continue;
                }
                for (int e = (int) first[i]; e < first[i + 1]; e++) {
                    Record r2 = db.recordAtRow(cand[e]);
                    for (MatchListener l : listeners) {
                        if (kind[e] == DukeHip.KIND_MATCH) l.matches(r1, r2, prob[e]);
                        else l.matchesPerhaps(r1, r2, prob[e]);
                    }
                }
            }
        } finally {
            DukeHip.freeResult(res);
        }
        for (MatchListener l : listeners) l.batchDone();
        if (db.indexingIsDisabled()) db.dropTransient();   // the batch never entered the index
    }

    /** Processor.compare(r1, r2) of any two records (indexed or not): dk_compare_values. */
    @Override
    public double compare(Record r1, Record r2) {
        return db.compareValues(r1, r2);
    }
}
