package io.sesam.dukemicroservice.gpu;

import java.util.ArrayList;
import java.util.Collection;
import java.util.List;

import io.sesam.dukemicroservice.SinceAwareInMemoryLinkDatabase;
import no.priv.garshol.duke.Link;
import no.priv.garshol.duke.LinkKind;
import no.priv.garshol.duke.LinkStatus;

/**
 * The pipeline's link database ("in-memory" link-database-type, App.java:571-574) held natively
 * (dk_linkdb) and written in bulk: GpuProcessor hands each batch's match arrays to
 * dk_linkdb_apply after the replay -- what BaseLinkDatabaseMatchListener's wrapped
 * LinkDatabaseMatchListener does per callback (BaseLinkDatabaseMatchListener.java:50,
 * 53-109) -- instead of one assertLink per link.  That per-callback path still runs (the
 * listener is unchanged), but GpuProcessor opens a listener window around each batch
 * (batchReady .. batchDone) in which every write reaching this database is dropped -- the
 * listener's INFERRED assertions and its own retractions of links a record no longer
 * produced alike -- so the bulk write alone changes the database, as the Python host's
 * GpuProcessor.set_link_database does (tests/test_linkdb.py::test_java_wiring_*).  Outside
 * the window the routes' writes stay: getChangesSince for the GET ?since= feed (App.java:742,
 * 843), getAllLinksFor + a retracted assertLink for deleted records (App.java:994-999,
 * dk_linkdb_retract).  Links carry record ID strings as in Duke; the
 * natives work on the database's interned IDs (GpuBlockingDatabase.ids()).
 */
public class GpuLinkDatabase extends SinceAwareInMemoryLinkDatabase {
    private final long ids;
    private final long db;
    private boolean nativeMode = true;   // false after handOver(): the Java superclass serves
    private boolean listenerWindow;      // GpuProcessor is inside a batch: listener writes dropped

    public GpuLinkDatabase(GpuBlockingDatabase database) {
        this.ids = database.ids();
        this.db = DukeHip.linkdbCreate(ids);
    }

    /** GpuProcessor, around a batch's batchReady .. batchDone: the per-callback listener's
     *  writes (assertLink of INFERRED and of RETRACTED links) are dropped while it is open. */
    void setListenerWindow(boolean open) {
        listenerWindow = open;
    }

    /** One batch's match list (dk_result arrays) for query records of the given IDs. */
    public long[] applyBatch(long[] queryIdent, long[] first, long[] candidateIdent, double[] prob,
                             byte[] kind, long timestamp) {
        return DukeHip.linkdbApply(db, queryIdent, first, candidateIdent, prob, kind, timestamp);
    }

    /** GpuProcessor's fall-back to stock Duke: the links move into the Java superclass (the
     *  reference's own SinceAwareInMemoryLinkDatabase), which the per-callback listener then
     *  writes as in the reference. */
    void handOver() {
        listenerWindow = false;
        if (!nativeMode) return;
        List<Link> all = getChangesSince(Long.MIN_VALUE);
        nativeMode = false;
        for (Link l : all) super.assertLink(l);
    }

    @Override
    public void assertLink(Link link) {
        if (!nativeMode) {
            super.assertLink(link);
            return;
        }
        // inside a batch: the listener's writes -- applyBatch has written (or will write) the
        // batch's links and retractions itself
        if (listenerWindow) return;
        // the deleted-record branch (App.java:994-999): link.retract() then assertLink, per link
        if (link.getStatus() == LinkStatus.RETRACTED) {
            long a = DukeHip.internerFind(ids, link.getID1()), b = DukeHip.internerFind(ids, link.getID2());
            if (a >= 0 && b >= 0) DukeHip.linkdbRetract(db, a, b, link.getTimestamp());
        }
        // an INFERRED link outside a batch: no route writes one (the listener runs only
        // inside deduplicate)
    }

    @Override
    public Collection<Link> getAllLinksFor(String id) {
        if (!nativeMode) return super.getAllLinksFor(id);
        long ident = DukeHip.internerFind(ids, id);
        return ident < 0 ? new ArrayList<Link>() : links(DukeHip.linkdbLinksFor(db, ident));
    }

    @Override
    public List<Link> getChangesSince(long since) {
        if (!nativeMode) return super.getChangesSince(since);
        return links(DukeHip.linkdbChangesSince(db, since));
    }

    private List<Link> links(long list) {
        try {
            long[] id1 = DukeHip.linkListId1(list), id2 = DukeHip.linkListId2(list);
            byte[] status = DukeHip.linkListStatus(list), kind = DukeHip.linkListKind(list);
            double[] conf = DukeHip.linkListConfidence(list);
            long[] ts = DukeHip.linkListTimestamp(list);
            List<Link> out = new ArrayList<>(id1.length);
            for (int i = 0; i < id1.length; i++)
                // [Duke 1.2, recalled] Link(id1, id2, status, kind, confidence, timestamp)
                out.add(new Link(DukeHip.internerString(ids, id1[i]), DukeHip.internerString(ids, id2[i]),
                                 status[i] == DukeHip.LINK_RETRACTED ? LinkStatus.RETRACTED : LinkStatus.INFERRED,
                                 kind[i] == DukeHip.LINK_SAME ? LinkKind.SAME : LinkKind.MAYBE, conf[i], ts[i]));
            return out;
        } finally {
            DukeHip.freeLinkList(list);
        }
    }

    @Override
    public void close() {
        DukeHip.linkdbDestroy(db);
    }
}
