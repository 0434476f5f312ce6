package io.sesam.dukemicroservice.gpu;

import java.util.ArrayList;
import java.util.Collection;
import java.util.List;

import no.priv.garshol.duke.Configuration;
import no.priv.garshol.duke.Database;
import no.priv.garshol.duke.Processor;
import no.priv.garshol.duke.Record;
import no.priv.garshol.duke.matchers.MatchListener;

/**
 * Processor whose matching loop runs on the GPU (Duke 1.2 Processor.deduplicate, called at
 * App.java:1005 / 1159).  One batch: batchReady, index + commit (dk_upsert; dk_upsert_transient
 * while indexing is disabled, App.java:1130-1132), dk_match, the callbacks replayed on this
 * thread in Duke's order (per query record in batch order its matches / matchesPerhaps in
 * candidate order, or noMatchFor), the batch's links written in bulk (GpuLinkDatabase), batchDone.
 * Mirrors dukehip/processor.py GpuProcessor.
 *
 * Stock-Duke fallback: a batch the GPU path cannot take (dk_upsert DK_E_UNSUPPORTED -- a
 * (Weighted)Levenshtein value over 256 code units, a Lucene lookup value outside Latin-1, a
 * second value for one property) hands the pipeline over to stock Duke for good: the
 * `fallback` database (the reference's own IncrementalLuceneDatabase, configured as
 * App.configureDatabase does) is filled with every record the GPU index holds, the batch runs
 * on a stock Processor with the same listeners, and so do all later batches.  The GPU index
 * is left as it was (dk_upsert is failure-atomic), so no batch is half-applied.
 */
public class GpuProcessor extends Processor {
    /** Creates the stock database the pipeline falls back to (App.java:329-342 / 450-463). */
    public interface FallbackDatabase {
        Database create();
    }

    private final Configuration config;
    private final GpuBlockingDatabase db;
    private final List<MatchListener> listeners = new ArrayList<>();
    private final FallbackDatabase fallback;
    private GpuLinkDatabase links;
    private GpuJdbcLinkDatabase jdbcLinks;   // the opt-in H2 bulk writer (DUKEHIP_H2_BULK)
    private Processor stock;   // non-null once the pipeline has fallen back

    public GpuProcessor(Configuration config, GpuBlockingDatabase db, FallbackDatabase fallback) {
        super(config, false);
        this.config = config;
        this.db = db;
        this.fallback = fallback;
    }

    /** The pipeline's link database, written in bulk after each batch (not while indexing is
     *  disabled: App.java:1131-1132 disables the link writes of httptransform batches). */
    public void setLinkDatabase(GpuLinkDatabase links) {
        this.links = links;
    }

    /** The H2 link database with bulk writes (opt-in, GpuJdbcLinkDatabase): the same
     *  listener window, the batch's links written by one MERGE batch per deduplicate. */
    public void setJdbcLinkDatabase(GpuJdbcLinkDatabase links) {
        this.jdbcLinks = links;
    }

    private void window(boolean open) {
        if (links != null) links.setListenerWindow(open);
        if (jdbcLinks != null) jdbcLinks.setListenerWindow(open);
    }

    @Override
    public void addMatchListener(MatchListener listener) {
        super.addMatchListener(listener);
        listeners.add(listener);
        if (stock != null) stock.addMatchListener(listener);
    }

    @Override
    public void deduplicate(Collection<Record> records) {
        if (stock != null) {
            stock.deduplicate(records);
            return;
        }
        List<Record> batch = new ArrayList<>(records);
        // records given to Database.index() beforehand (the deleted records of
        // App.java:988-1001, 1121-1137) are committed together with the batch
        List<Record> pending = db.takePending();
        List<Record> all = new ArrayList<>(pending);
        all.addAll(batch);
        int[] allRows;
        try {
            allRows = db.indexBatch(all, db.indexingIsDisabled());
        } catch (DukeHipException e) {
            if (e.code() != DukeHip.E_UNSUPPORTED || fallback == null) throw e;
            fallBack(pending).deduplicate(records);
            return;
        }
        int[] rows = new int[batch.size()];
        System.arraycopy(allRows, pending.size(), rows, 0, rows.length);
        window(true);
        try {
            for (MatchListener l : listeners) l.batchReady(batch.size());
            matchAndReplay(rows, batch);
            for (MatchListener l : listeners) l.batchDone();
        } finally {
            window(false);
        }
        db.releaseDeferred();
        if (db.indexingIsDisabled()) db.dropTransient();   // the batch never entered the index
    }

    /**
     * Processor.deduplicate of a POSTed body taken natively (dk_pack_json: no Gson tree and no
     * Record objects on the way in; the listeners get Records built for the rows they see).
     * Returns false -- nothing done -- when the native reader declines the body (lenient Gson
     * syntax, characters outside the native cleaners); the route then parses it as today.
     */
    public boolean deduplicateJson(byte[] body, GpuBlockingDatabase.JsonSource src) {
        if (stock != null) return false;
        List<Record> pending = db.takePending();
        if (!pending.isEmpty()) db.indexBatch(pending, false);
        int[] rows;
        try {
            rows = db.indexJson(body, src, db.indexingIsDisabled());
        } catch (DukeHipException e) {
            if (e.code() != DukeHip.E_UNSUPPORTED) throw e;
            return false;
        }
        window(true);
        try {
            for (MatchListener l : listeners) l.batchReady(rows.length);
            matchAndReplay(rows, null);
            for (MatchListener l : listeners) l.batchDone();
        } finally {
            window(false);
        }
        db.releaseDeferred();
        if (db.indexingIsDisabled()) db.dropTransient();
        return true;
    }

    private void matchAndReplay(int[] rows, List<Record> batch) {
        long res = DukeHip.match(db.ctx(), rows);
        try {
            long[] first = DukeHip.resultFirst(res);
            int[] cand = DukeHip.resultCandidate(res);
            double[] prob = DukeHip.resultProb(res);
            byte[] kind = DukeHip.resultKind(res);
            if (!listeners.isEmpty()) {
                for (int i = 0; i < rows.length; i++) {
                    Record r1 = batch != null ? batch.get(i) : db.recordAtRow(rows[i]);
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
            }
            if (links != null && !db.indexingIsDisabled()) {
                long[] qid = new long[rows.length], cid = new long[cand.length];
                for (int i = 0; i < rows.length; i++) qid[i] = db.identAtRow(rows[i]);
                for (int e = 0; e < cand.length; e++) cid[e] = db.identAtRow(cand[e]);
                links.applyBatch(qid, first, cid, prob, kind, System.currentTimeMillis());
            }
            if (jdbcLinks != null && !db.indexingIsDisabled()) {
                String[] qs = new String[rows.length], cs = new String[cand.length];
                for (int i = 0; i < rows.length; i++) qs[i] = DukeHip.internerString(db.ids(), db.identAtRow(rows[i]));
                for (int e = 0; e < cand.length; e++) cs[e] = DukeHip.internerString(db.ids(), db.identAtRow(cand[e]));
                jdbcLinks.applyBatch(qs, first, cs, prob, kind, System.currentTimeMillis());
            }
        } finally {
            DukeHip.freeResult(res);
        }
    }

    /** The hand-over to stock Duke: every record the GPU index holds (plus the records that
     *  were pending) into the fallback database, then a stock Processor over it. */
    private Processor fallBack(List<Record> pending) {
        Database stockDb = fallback.create();
        for (Record r : db.liveRecords()) stockDb.index(r);
        for (Record r : pending) stockDb.index(r);
        stockDb.commit();
        config.setDatabase(stockDb);
        if (links != null) links.handOver();   // the listener writes links per callback again
        jdbcLinks = null;                      // (the H2 table: per callback, as in the reference)
        stock = new Processor(config, false);
        for (MatchListener l : listeners) stock.addMatchListener(l);
        return stock;
    }

    /** Processor.compare(r1, r2) of any two records (indexed or not): dk_compare_values. */
    @Override
    public double compare(Record r1, Record r2) {
        return stock != null ? stock.compare(r1, r2) : db.compareValues(r1, r2);
    }

    @Override
    public Database getDatabase() {
        return stock != null ? stock.getDatabase() : db;
    }
}
